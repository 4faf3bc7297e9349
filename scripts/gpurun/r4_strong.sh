#!/bin/bash
# round 4: config 4's strong share (512 envs/GPU): rollout workgroup shapes A/B, step-kernel block, update trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/strong_ab.jsonl
for w in 8 4 1; do
  echo "{\"wpg\": $w}" >> gpurun_out/strong_ab.jsonl
  DGPPO_ROLLOUT_WPG=$w timeout -k 10 300 python -u scripts/config_bench.py --only x512 --no-ppo >> gpurun_out/strong_ab.jsonl 2>> gpurun_out/strong_ab.err || exit $?
done
echo '{"step_kernel": "block"}' >> gpurun_out/strong_ab.jsonl
timeout -k 10 300 python -u scripts/config_bench.py --only x512 --no-ppo --step-kernel block >> gpurun_out/strong_ab.jsonl 2>> gpurun_out/strong_ab.err || exit $?
cat gpurun_out/strong_ab.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/strong_trace -o run --output-format csv -- python3 scripts/update_time.py --env LidarBicycleTarget --envs 512 --batch 2048 --reps 3 > gpurun_out/strong_trace.log 2>&1 || exit $?
f=$(ls gpurun_out/strong_trace/*/*kernel_trace.csv 2>/dev/null | head -n 1)
[ -n "$f" ] && python3 scripts/busy.py "$f" 2000000 > gpurun_out/strong_busy.txt
tail -n 12 gpurun_out/strong_busy.txt
echo done

#!/bin/bash
# round 4: where the n = 32 update's time goes (LidarSpread n32 o8, 1024 envs, batch 16384)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/n32
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_update_gpu.py tests/test_update_dynamics_gpu.py tests/test_informarl_gpu.py -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider -x > gpurun_out/n32/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 3 gpurun_out/n32/tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  DGPPO_PHASE_EVENTS=1 timeout -k 10 240 python -u scripts/update_time.py >> gpurun_out/n32/time.jsonl 2>&1 || exit $?
done
DGPPO_PHASE_EVENTS=1 timeout -k 10 300 python -u scripts/update_time.py -n 32 --obs 8 --envs 1024 --reps 3 >> gpurun_out/n32/time.jsonl 2>&1 || exit $?
cat gpurun_out/n32/time.jsonl
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/n32/prof -o run --output-format csv -- python3 scripts/update_time.py -n 32 --obs 8 --envs 1024 --reps 2 > gpurun_out/n32/prof.log 2>&1 || exit $?
f=$(ls gpurun_out/n32/prof/*kernel_stats.csv gpurun_out/n32/prof/*/*kernel_stats.csv 2>/dev/null | head -n 1)
python3 scripts/top_kernels.py "$f" 25
rm -f gpurun_out/n32/prof/*kernel_trace.csv gpurun_out/n32/prof/*/*kernel_trace.csv

#!/bin/bash
# round 4: small-K GEMM kernel (tests + A/B); policy rollouts split into env slices on 2 / 4 streams
# (DGPPO_ROLLOUT_LANES) -- collect and update
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gemm_epi_gpu.py tests/test_nets_gpu.py -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider -x > gpurun_out/lanes_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 3 gpurun_out/lanes_tests.log; [ $rc -ne 0 ] && exit $rc
: > gpurun_out/lanes.jsonl
for k in 1 0; do
  DGPPO_GEMM_SMALLK=$k DGPPO_PHASE_EVENTS=1 timeout -k 10 240 python -u scripts/update_time.py >> gpurun_out/lanes.jsonl 2>> gpurun_out/lanes.err || exit $?
done
for l in 1 2 4 1 2; do
  DGPPO_ROLLOUT_LANES=$l DGPPO_PHASE_EVENTS=1 timeout -k 10 240 python -u scripts/update_time.py >> gpurun_out/lanes.jsonl 2>> gpurun_out/lanes.err || exit $?
done
for l in 1 2; do
  DGPPO_ROLLOUT_LANES=$l DGPPO_PHASE_EVENTS=1 timeout -k 10 240 python -u scripts/update_time.py --env LidarBicycleTarget --envs 512 --batch 2048 >> gpurun_out/lanes.jsonl 2>> gpurun_out/lanes.err || exit $?
done
cat gpurun_out/lanes.jsonl

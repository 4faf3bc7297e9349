#!/bin/bash
# Weight-gradient GEMM variants (DGPPO_WGRAD_FLAT branch-free loads, DGPPO_WGRAD_U row pairs in flight): per-shape
# times (scripts/gemm_bench.py), then parity tests and the update.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for k in "DGPPO_WGRAD_FLAT=0" "DGPPO_WGRAD_FLAT=1" "DGPPO_WGRAD_FLAT=1 DGPPO_WGRAD_U=4"; do
  echo "== $k"; env $k SHAPE=wgrad timeout -k 10 120 python3 scripts/gemm_bench.py || exit 1
done
timeout -k 10 300 python -u -m pytest tests/test_nets_gpu.py tests/test_update_gpu.py -m gpu -x -q --timeout 180 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/wg_tests.log 2>&1; rc=$?; tail -3 gpurun_out/wg_tests.log; [ $rc -eq 0 ] || exit $rc
for k in "DGPPO_WGRAD_FLAT=1" "DGPPO_WGRAD_FLAT=0" "DGPPO_WGRAD_FLAT=1 DGPPO_WGRAD_U=4"; do
  env $k DGPPO_PHASE_EVENTS=1 timeout -k 10 300 python3 scripts/update_time.py --reps 5 || exit 1
done

#!/bin/bash
# Update-parity tests, then the update time with the weight-gradient GEMMs on side streams (DGPPO_WGRAD_SIDE=1) vs
# inline (=0), interleaved on one box: the bench config and config 4's per-rank share.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_update_gpu.py tests/test_update_dynamics_gpu.py tests/test_distributed_gpu.py \
  -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/wside_tests.log 2>&1
rc=$?; tail -3 gpurun_out/wside_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for f in 1 0; do
    DGPPO_WGRAD_SIDE=$f timeout -k 10 200 python3 scripts/update_time.py --reps 5 | sed "s/^/side=$f 4096: /" || exit 1
    DGPPO_WGRAD_SIDE=$f timeout -k 10 200 python3 scripts/update_time.py --envs 512 --batch 2048 --env LidarBicycleTarget \
      --reps 5 | sed "s/^/side=$f c4: /" || exit 1
  done
done

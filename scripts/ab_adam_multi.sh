#!/bin/bash
# dgppo_adam_multi (DGPPO_ADAM_MULTI=1, default) vs the per-net grad_norm + adam pairs: parity tests, then the update
# time at the bench config and at config 4's per-rank share (2048-sample minibatches replayed from hipGraphs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_adam_multi_gpu.py tests/test_update_gpu.py tests/test_update_dynamics_gpu.py -m gpu -x -q \
  --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/am_tests.log 2>&1; rc=$?
tail -3 gpurun_out/am_tests.log; [ $rc -eq 0 ] || exit $rc
for args in "" "--env LidarBicycleTarget --envs 512 --batch 2048"; do
  for i in 1 2; do
    for k in 1 0; do
      DGPPO_ADAM_MULTI=$k DGPPO_PHASE_EVENTS=1 timeout -k 10 300 python3 scripts/update_time.py $args --reps 5 2>/dev/null | \
        python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('multi=$k $args', d['collect_ms'], d['update_ms'], d['phases_ms'])" || exit 1
    done
  done
done

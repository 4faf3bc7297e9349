#!/bin/bash
# Stream lanes: rollout parity tests, then the env-only bench (DGPPO_BENCH_LANES) and the DGPPO
# collect/update (DGPPO_ROLLOUT_LANES) with 1 and 2 lanes.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_rollout_gpu.py -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/lanes_tests.log 2>&1
tail -2 gpurun_out/lanes_tests.log
B="python bench.py --steps 5 --warmup 2 --ppo-iters 3 --no-cpu-baseline"
for L in 1 2 1 2; do
  DGPPO_ROLLOUT_LANES=$L timeout -k 10 240 $B > gpurun_out/plan_$L.log 2>&1
  echo "rollout_lanes=$L $(tail -1 gpurun_out/plan_$L.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['ppo']; print(d['value'], p['collect_ms'], p['update_ms'], p['updates_per_s'])")"
done

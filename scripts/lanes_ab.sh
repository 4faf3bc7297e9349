#!/bin/bash
# A/B of the env-only rollout stepped as 1 / 2 / 4 env slices on separate streams (bench.py,
# DGPPO_BENCH_LANES), after the lanes parity test.
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_rollout_gpu.py -m gpu -x -v --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/lanes_tests.log 2>&1
B="python bench.py --steps 20 --warmup 3 --ppo-iters 0 --no-cpu-baseline"
for L in 1 2 4 1 2 4; do
  DGPPO_BENCH_LANES=$L timeout -k 10 180 $B > gpurun_out/lanes_$L.log 2>&1
  echo "lanes=$L $(tail -1 gpurun_out/lanes_$L.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done
tail -2 gpurun_out/lanes_tests.log

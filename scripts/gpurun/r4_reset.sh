#!/bin/bash
# round 4: bitmask rejection sampler in the env reset: env / rollout / variant tests (bit-exact), reset timing,
# episodes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_env_gpu.py tests/test_rollout_gpu.py tests/test_env_variants_gpu.py tests/test_train_gpu.py -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider -x > gpurun_out/reset_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 4 gpurun_out/reset_tests.log
[ $rc -ne 0 ] && exit $rc
: > gpurun_out/reset_time2.jsonl
for e in "LidarSpread -n 8 --obs 3" "LidarBicycleTarget -n 8 --obs 3" "MPESpread -n 3 --obs 3"; do
  timeout -k 10 120 python -u scripts/reset_time.py --env $e >> gpurun_out/reset_time2.jsonl 2>/dev/null || exit $?
done
cat gpurun_out/reset_time2.jsonl
timeout -k 10 300 python -u scripts/config_bench.py --only "x512" --no-ppo > gpurun_out/reset_cb.jsonl 2>/dev/null || exit $?
timeout -k 10 300 python -u scripts/config_bench.py --only "LidarSpread n8" --no-ppo >> gpurun_out/reset_cb.jsonl 2>/dev/null || exit $?
timeout -k 10 300 python -u scripts/config_bench.py --only "MPESpread" --no-ppo >> gpurun_out/reset_cb.jsonl 2>/dev/null || exit $?
cat gpurun_out/reset_cb.jsonl
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --ppo-iters 0 > gpurun_out/reset_bench.json 2>/dev/null || exit $?
tail -c 400 gpurun_out/reset_bench.json

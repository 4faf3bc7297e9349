#!/bin/bash
# round 4: parallel reset draws (env tests + reset timing), minibatch hipGraph replay at the bench's 16384-sample
# minibatches (A/B)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_env_gpu.py tests/test_rollout_gpu.py tests/test_env_variants_gpu.py -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider -x > gpurun_out/gb_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 4 gpurun_out/gb_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -u scripts/reset_time.py > gpurun_out/reset_time.jsonl 2>&1 || exit $?
timeout -k 10 120 python -u scripts/reset_time.py --env LidarBicycleTarget >> gpurun_out/reset_time.jsonl 2>&1 || exit $?
timeout -k 10 120 python -u scripts/reset_time.py --env MPESpread -n 3 --obs 3 >> gpurun_out/reset_time.jsonl 2>&1 || exit $?
cat gpurun_out/reset_time.jsonl
: > gpurun_out/graphbig.jsonl
for g in 1 0 1 0; do
  DGPPO_UPDATE_GRAPH=$g timeout -k 10 240 python -u scripts/update_time.py >> gpurun_out/graphbig.jsonl 2>> gpurun_out/graphbig.err || exit $?
done
cat gpurun_out/graphbig.jsonl

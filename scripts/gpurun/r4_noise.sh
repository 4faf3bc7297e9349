#!/bin/bash
# round 4: in-kernel policy noise (ABI 10) + adaptive rollout workgroup size: suite, collect / update timing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider -x > gpurun_out/noise_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 6 gpurun_out/noise_tests.log
[ $rc -ne 0 ] && exit $rc
: > gpurun_out/noise_ab.jsonl
timeout -k 10 240 python -u scripts/update_time.py >> gpurun_out/noise_ab.jsonl 2>> gpurun_out/noise_ab.err || exit $?
timeout -k 10 240 python -u scripts/update_time.py --env LidarBicycleTarget --envs 512 --batch 2048 >> gpurun_out/noise_ab.jsonl 2>> gpurun_out/noise_ab.err || exit $?
timeout -k 10 300 python -u scripts/config_bench.py --only x512 --reps 3 >> gpurun_out/noise_ab.jsonl 2>> gpurun_out/noise_ab.err || exit $?
cat gpurun_out/noise_ab.jsonl

#!/bin/bash
# round 4: GRU kernels with register-resident Wh fragments: bit-identity + parity tests, update A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gru_form_gpu.py tests/test_nets_gpu.py tests/test_update_dynamics_gpu.py tests/test_update_gpu.py -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider -x > gpurun_out/gru_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 4 gpurun_out/gru_tests.log
[ $rc -ne 0 ] && exit $rc
: > gpurun_out/gru_ab.jsonl
for r in 1 0 1 0; do
  DGPPO_GRU_REGB=$r DGPPO_PHASE_EVENTS=1 timeout -k 10 240 python -u scripts/update_time.py >> gpurun_out/gru_ab.jsonl 2>> gpurun_out/gru_ab.err || exit $?
done
for r in 1 0; do
  DGPPO_GRU_REGB=$r DGPPO_PHASE_EVENTS=1 timeout -k 10 240 python -u scripts/update_time.py --env LidarBicycleTarget --envs 512 --batch 2048 >> gpurun_out/gru_ab.jsonl 2>> gpurun_out/gru_ab.err || exit $?
done
cat gpurun_out/gru_ab.jsonl

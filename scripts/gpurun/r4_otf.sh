#!/bin/bash
# round 4: graph-form forward with on-the-fly hit rows (n = 32): parity + bit-identity tests, n = 32 A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/otf
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_nets_gpu.py tests/test_attn_gm_gpu.py tests/test_rollout_gpu.py -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider -x > gpurun_out/otf/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 3 gpurun_out/otf/tests.log; [ $rc -ne 0 ] && exit $rc
: > gpurun_out/otf/ab.jsonl
for o in 1 1; do
  DGPPO_ATTN_GRAPH_OTF=$o DGPPO_PHASE_EVENTS=1 timeout -k 10 300 python -u scripts/update_time.py -n 32 --obs 8 --envs 1024 --reps 3 >> gpurun_out/otf/ab.jsonl 2>> gpurun_out/otf/ab.err || exit $?
done
cat gpurun_out/otf/ab.jsonl

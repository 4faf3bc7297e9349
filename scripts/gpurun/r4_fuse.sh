#!/bin/bash
# round 4: the fused GEMM epilogues on the GPU: epilogue tests, the network / update parity suites, then the update
# time with DGPPO_FUSE_LN=1 vs 0 interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider -x > gpurun_out/fuse_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -25 gpurun_out/fuse_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
: > gpurun_out/fuse_ab.jsonl
for k in 1 0 1 0; do
  DGPPO_FUSE_LN=$k timeout -k 10 240 python -u scripts/update_time.py >> gpurun_out/fuse_ab.jsonl 2>> gpurun_out/fuse_ab.err || exit $?
done
cat gpurun_out/fuse_ab.jsonl
exit $rc

#!/bin/bash
# round 4: LayerNorm-backward epilogue reading the forward's stored statistics; suite, update A/B, kernel stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider -x > gpurun_out/fuse4_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 6 gpurun_out/fuse4_tests.log
[ $rc -ne 0 ] && exit $rc
: > gpurun_out/fuse4_ab.jsonl
for k in 1 0 1 0; do
  DGPPO_FUSE_LN=$k timeout -k 10 240 python -u scripts/update_time.py >> gpurun_out/fuse4_ab.jsonl 2>> gpurun_out/fuse4_ab.err || exit $?
done
cat gpurun_out/fuse4_ab.jsonl
for k in 1 0; do
  DGPPO_FUSE_LN=$k timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fuse4_prof$k -o run -- python3 scripts/update_time.py > gpurun_out/fuse4_prof$k.log 2>&1 || exit $?
done
echo done

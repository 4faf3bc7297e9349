#!/bin/bash
# round 4: full GPU suite on the fused-epilogue + split-graph build, update A/B (fused LN on / off), config 4 shares
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider -x > gpurun_out/fuse3_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -6 gpurun_out/fuse3_tests.log
[ $rc -ne 0 ] && exit $rc
: > gpurun_out/fuse3_ab.jsonl
for k in 1 0 1 0; do
  DGPPO_FUSE_LN=$k timeout -k 10 240 python -u scripts/update_time.py >> gpurun_out/fuse3_ab.jsonl 2>> gpurun_out/fuse3_ab.err || exit $?
done
for g in 1 0; do
  DGPPO_UPDATE_GRAPH=$g timeout -k 10 240 python -u scripts/update_time.py --env LidarBicycleTarget --envs 512 --batch 2048 >> gpurun_out/fuse3_ab.jsonl 2>> gpurun_out/fuse3_ab.err || exit $?
done
timeout -k 10 240 python -u scripts/update_time.py --env LidarBicycleTarget --envs 4096 --batch 16384 >> gpurun_out/fuse3_ab.jsonl 2>> gpurun_out/fuse3_ab.err || exit $?
cat gpurun_out/fuse3_ab.jsonl

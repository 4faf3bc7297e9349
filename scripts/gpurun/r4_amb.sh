#!/bin/bash
# round 4: Vl's top-layer ReLU backward fused into the agent-mean broadcast; full GPU suite + update timing
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider -x > gpurun_out/amb_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 4 gpurun_out/amb_tests.log
[ $rc -ne 0 ] && exit $rc
: > gpurun_out/amb.jsonl
for k in 1 0; do
  DGPPO_FUSE_LN=$k timeout -k 10 240 python -u scripts/update_time.py >> gpurun_out/amb.jsonl 2>> gpurun_out/amb.err || exit $?
done
cat gpurun_out/amb.jsonl
DGPPO_PHASE_EVENTS=1 timeout -k 10 240 python -u scripts/update_time.py >> gpurun_out/amb.jsonl 2>> gpurun_out/amb.err || exit $?
DGPPO_PHASE_EVENTS=1 timeout -k 10 240 python -u scripts/update_time.py --env LidarBicycleTarget --envs 512 --batch 2048 >> gpurun_out/amb.jsonl 2>> gpurun_out/amb.err || exit $?
tail -n 2 gpurun_out/amb.jsonl

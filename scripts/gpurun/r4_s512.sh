#!/bin/bash
# round 4: stream overlap at config 4's 512-env share (graph replay on), streams on / off
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/s512.jsonl
for st in 1 0; do
  DGPPO_STREAMS=$st DGPPO_PHASE_EVENTS=1 timeout -k 10 240 python -u scripts/update_time.py --env LidarBicycleTarget --envs 512 --batch 2048 >> gpurun_out/s512.jsonl 2>> gpurun_out/s512.err || exit $?
done
cat gpurun_out/s512.jsonl

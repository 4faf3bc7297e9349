#!/bin/bash
# round 4: do the update's three streams overlap?  HW queues per process (HIP default 4) vs 8 / 16, and streams off
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
: > gpurun_out/hwq_ab.jsonl
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 240 python -u scripts/update_time.py >> gpurun_out/hwq_ab.jsonl 2>> gpurun_out/hwq_ab.err || exit $?
  echo "{\"hwq\": $q}" >> gpurun_out/hwq_ab.jsonl
done
DGPPO_STREAMS=0 timeout -k 10 240 python -u scripts/update_time.py >> gpurun_out/hwq_ab.jsonl 2>> gpurun_out/hwq_ab.err || exit $?
echo '{"streams": 0}' >> gpurun_out/hwq_ab.jsonl
for q in 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 240 python -u scripts/update_time.py --env LidarBicycleTarget --envs 512 --batch 2048 >> gpurun_out/hwq_ab.jsonl 2>> gpurun_out/hwq_ab.err || exit $?
  echo "{\"hwq\": $q, \"x512\": 1}" >> gpurun_out/hwq_ab.jsonl
done
cat gpurun_out/hwq_ab.jsonl
bash scripts/gpurun/r4_strong.sh

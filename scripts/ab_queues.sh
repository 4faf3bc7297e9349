#!/bin/bash
# Hardware queues per process (GPU_MAX_HW_QUEUES, HIP's default 4) x rollout lanes (DGPPO_ROLLOUT_LANES): collect and
# update time at the bench config (scripts/update_time.py), one process per setting.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for q in 4 8 16; do
  for l in 1 2 4; do
    GPU_MAX_HW_QUEUES=$q DGPPO_ROLLOUT_LANES=$l DGPPO_PHASE_EVENTS=1 timeout -k 10 300 python3 scripts/update_time.py --reps 5 \
      > gpurun_out/q_${q}_${l}.json 2>gpurun_out/q.err || { tail -5 gpurun_out/q.err; exit 1; }
    echo "queues=$q lanes=$l $(python3 -c "import json;d=json.load(open('gpurun_out/q_${q}_${l}.json'));print(d['collect_ms'], d['update_ms'], d['phases_ms'])")"
  done
done

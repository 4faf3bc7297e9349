#!/bin/bash
# config 4's per-rank share: phase split (DGPPO_PHASE_EVENTS) of the 512-env update and its kernel list per minibatch
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
DGPPO_PHASE_EVENTS=1 timeout -k 10 200 python3 scripts/update_time.py --env LidarBicycleTarget --envs 512 --batch 2048 --reps 3 2>/dev/null | tail -1 || exit 1
DGPPO_PHASE_EVENTS=1 timeout -k 10 200 python3 scripts/update_time.py --reps 3 2>/dev/null | tail -1 || exit 1
bash scripts/r06_c4_trace.sh

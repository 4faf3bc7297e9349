#!/bin/bash
# Kernel trace of config 4's per-rank update share (LidarBicycleTarget n8 o3, 512 envs, 2048-sample minibatches).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c4 -o run -- \
  python3 scripts/update_time.py --env LidarBicycleTarget --envs 512 --batch 2048 --reps 1 > gpurun_out/c4.log 2>&1 || { tail gpurun_out/c4.log; exit 1; }
python3 scripts/mb_gaps.py gpurun_out/c4

#!/bin/bash
# Interleaved A/B of two env-kernel builds on one box: the in-tree library against
# dgppo_fov_amd/lib/libdgppo_hip_prev.so (built by hand from an older env_step.hip), LidarSpread n=8
# episodes (reset + 128 steps, scripts/config_bench.py), 3 runs each -> gpurun_out/ab_{new,prev}.txt.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for i in 1 2 3; do
  timeout -k 10 100 python -u scripts/config_bench.py --only "LidarSpread n8" --no-ppo >> gpurun_out/ab_new.txt 2>/dev/null || exit 1
  DGPPO_HIP_LIB=$PWD/dgppo_fov_amd/lib/libdgppo_hip_prev.so timeout -k 10 100 \
    python -u scripts/config_bench.py --only "LidarSpread n8" --no-ppo >> gpurun_out/ab_prev.txt 2>/dev/null || exit 1
done

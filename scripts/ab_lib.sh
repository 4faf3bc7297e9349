#!/bin/bash
# Interleaved A/B of the in-tree library against dgppo_fov_amd/lib/libdgppo_hip_prev.so on scripts/ab_passes.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for i in 1 2 3; do
  timeout -k 10 120 python3 scripts/ab_passes.py || exit 1
  DGPPO_HIP_LIB=$PWD/dgppo_fov_amd/lib/libdgppo_hip_prev.so timeout -k 10 120 python3 scripts/ab_passes.py || exit 1
done

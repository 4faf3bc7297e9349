#!/bin/bash
# per-pass kernel split of three library builds (current, _attn, _prev), twice, interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=$PWD/dgppo_fov_amd/lib
KNOBS="DGPPO_X=0,DGPPO_HIP_LIB=$L/libdgppo_hip_attn.so,DGPPO_HIP_LIB=$L/libdgppo_hip_prev.so,DGPPO_X=1,DGPPO_HIP_LIB=$L/libdgppo_hip_attn.so,DGPPO_HIP_LIB=$L/libdgppo_hip_prev.so" \
  bash scripts/prof_mb2.sh | grep -E "===|gnn_layer|attn_bwd2r" || exit 1

#!/bin/bash
# fused layer forward raw-row staging modes (DGPPO_LAYER_STAGE 0 / 1 / 2): per-pass kernel split
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
KNOBS="DGPPO_LAYER_STAGE=0,DGPPO_LAYER_STAGE=1,DGPPO_LAYER_STAGE=2" bash scripts/prof_mb2.sh | grep -E "===|==|gnn_layer" || exit 1

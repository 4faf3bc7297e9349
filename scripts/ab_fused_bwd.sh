#!/bin/bash
# The fused layer backward (DGPPO_FUSED_LAYER_BWD=1; gather form, or DGPPO_LAYER_BWD_STAGE=1 staged graphs) against
# attn_bwd2r + GEMMs: parity tests, per-pass kernels, update time.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gnn_layer_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/fb_tests.log 2>&1; rc=$?; tail -3 gpurun_out/fb_tests.log; [ $rc -eq 0 ] || exit $rc
KNOBS="DGPPO_FUSED_LAYER_BWD=1,DGPPO_FUSED_LAYER_BWD=0" bash scripts/prof_mb2.sh | grep -E "===|==|bwd_kernel|attn_bwd" || exit 1
for k in "DGPPO_FUSED_LAYER_BWD=1" "DGPPO_FUSED_LAYER_BWD=0"; do
  env $k DGPPO_PHASE_EVENTS=1 timeout -k 10 300 python3 scripts/update_time.py --reps 5 || exit 1
done

#!/bin/bash
# Fused GraphTransformer layer forward / backward (ABI 11): parity tests, then per-pass minibatch kernels and the
# update with DGPPO_FUSED_LAYER=1 (LDS-loop and DPP weighted sums) vs 0 on one box.  TESTS overrides the tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gnn_layer_gpu.py tests/test_nets_gpu.py} -m gpu -x -q --timeout 180 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/fl_tests.log 2>&1
rc=$?; tail -5 gpurun_out/fl_tests.log; [ $rc -eq 0 ] || exit $rc
KNOBS="DGPPO_FUSED_LAYER=1,DGPPO_LAYER_WSUM=dpp,DGPPO_FUSED_LAYER=0" bash scripts/prof_mb2.sh || exit 1
rm -f gpurun_out/fl_update.jsonl
for k in "DGPPO_FUSED_LAYER=1" "DGPPO_LAYER_WSUM=dpp" "DGPPO_FUSED_LAYER=0"; do
  env $k DGPPO_PHASE_EVENTS=1 timeout -k 10 300 python3 scripts/update_time.py --reps 5 >> gpurun_out/fl_update.jsonl 2>gpurun_out/fl_update.err || exit 1
done
cat gpurun_out/fl_update.jsonl

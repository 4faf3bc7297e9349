#!/bin/bash
# Fused GraphTransformer layer forward (ABI 11): parity tests, then per-pass minibatch timing and the update with
# DGPPO_FUSED_LAYER=1 vs 0 interleaved on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gnn_layer_gpu.py tests/test_nets_gpu.py -m gpu -x -q --timeout 180 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/fl_tests.log 2>&1
rc=$?; tail -5 gpurun_out/fl_tests.log; [ $rc -eq 0 ] || exit $rc
for k in 1 0 1 0; do
  DGPPO_FUSED_LAYER=$k timeout -k 10 200 python3 scripts/mb_profile.py > gpurun_out/fl_mb_$k.txt 2>&1 || exit 1
  echo "fused=$k"; cat gpurun_out/fl_mb_$k.txt
done
for k in 1 0; do
  DGPPO_FUSED_LAYER=$k DGPPO_PHASE_EVENTS=1 timeout -k 10 300 python3 scripts/update_time.py --reps 5 >> gpurun_out/fl_update.jsonl 2>gpurun_out/fl_update.err || exit 1
done
cat gpurun_out/fl_update.jsonl

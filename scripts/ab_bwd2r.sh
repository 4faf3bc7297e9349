#!/bin/bash
# attn_bwd2r block staging (loads batched, optional next-block prefetch DGPPO_BWD2R_PF=1) against the previous build
# (dgppo_fov_amd/lib/libdgppo_hip_prev.so): parity tests, interleaved pass timings, per-kernel split.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_nets_gpu.py tests/test_gnn_layer_gpu.py tests/test_update_gpu.py -m gpu -x -q \
  --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/b2_tests.log 2>&1; rc=$?
tail -3 gpurun_out/b2_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 120 python3 scripts/ab_passes.py || exit 1
  DGPPO_BWD2R_PF=1 timeout -k 10 120 python3 scripts/ab_passes.py || exit 1
  DGPPO_HIP_LIB=$PWD/dgppo_fov_amd/lib/libdgppo_hip_prev.so timeout -k 10 120 python3 scripts/ab_passes.py || exit 1
done
KNOBS="DGPPO_BWD2R_PF=0,DGPPO_BWD2R_PF=1" bash scripts/prof_mb2.sh | grep -E "===|==|attn_bwd2r" || exit 1
for k in "DGPPO_BWD2R_PF=0" "DGPPO_BWD2R_PF=1"; do
  env $k DGPPO_PHASE_EVENTS=1 timeout -k 10 300 python3 scripts/update_time.py --reps 5 || exit 1
done

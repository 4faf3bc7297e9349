#!/bin/bash
# The in-tree library against the previous build (dgppo_fov_amd/lib/libdgppo_hip_prev.so): parity tests ($TESTS),
# interleaved pass timings (scripts/ab_passes.py), the minibatch kernel split and the update time of both.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TESTS=${TESTS:-"tests/test_nets_gpu.py tests/test_gnn_layer_gpu.py tests/test_update_gpu.py"}
timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/ab_tests.log 2>&1; rc=$?
tail -3 gpurun_out/ab_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 120 python3 scripts/ab_passes.py || exit 1
  DGPPO_HIP_LIB=$PWD/dgppo_fov_amd/lib/libdgppo_hip_prev.so timeout -k 10 120 python3 scripts/ab_passes.py || exit 1
done
KNOBS="DGPPO_X=0,DGPPO_HIP_LIB=$PWD/dgppo_fov_amd/lib/libdgppo_hip_prev.so" bash scripts/prof_mb2.sh | grep -E "===|==|${KGREP:-attn_bwd2r|gnn_layer}" || exit 1
for k in "DGPPO_X=0" "DGPPO_HIP_LIB=$PWD/dgppo_fov_amd/lib/libdgppo_hip_prev.so"; do
  env $k DGPPO_PHASE_EVENTS=1 timeout -k 10 300 python3 scripts/update_time.py --reps 5 || exit 1
done

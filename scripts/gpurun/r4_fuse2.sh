#!/bin/bash
# round 4: fused LayerNorm backward with the in-kernel column reduction: parity suites, update A/B, config 4 shares
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gemm_epi_gpu.py tests/test_nets_gpu.py tests/test_update_gpu.py tests/test_update_dynamics_gpu.py tests/test_informarl_lagr_gpu.py -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider -x > gpurun_out/fuse2_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -6 gpurun_out/fuse2_tests.log
[ $rc -ne 0 ] && exit $rc
: > gpurun_out/fuse2_ab.jsonl
for k in 1 0 1 0; do
  DGPPO_FUSE_LN=$k timeout -k 10 240 python -u scripts/update_time.py >> gpurun_out/fuse2_ab.jsonl 2>> gpurun_out/fuse2_ab.err || exit $?
done
cat gpurun_out/fuse2_ab.jsonl
bash scripts/gpurun/r4_cfg4.sh

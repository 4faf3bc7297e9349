#!/bin/bash
# round 6: wgrad A/B on the gemm_bench wgrad shapes (in-kernel partial reduction vs the second launch) + tests
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
: > gpurun_out/wgrad_ab.txt
TLIM=${TLIM:-300} TESTS="${TESTS:-tests/test_gemm_wgrad_gpu.py}" bash scripts/gpu_tests.sh || exit 1
for it in 1 2; do
  for cfg in ${CFGS:-"DGPPO_WGRAD_FUSED_REDUCE=1" "DGPPO_WGRAD_FUSED_REDUCE=0"}; do
    for r in 16384 131072; do
      echo "== $cfg ROWS=$r run $it" >> gpurun_out/wgrad_ab.txt
      env $cfg ROWS=$r SHAPE=wgrad timeout -k 10 120 python -u scripts/gemm_bench.py 2>/dev/null >> gpurun_out/wgrad_ab.txt || exit 1
    done
  done
done
cat gpurun_out/wgrad_ab.txt

#!/bin/bash
# round 6: wgrad tree epilogue: tests + gemm_bench wgrad shapes + update A/B (defer on)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TLIM=${TLIM:-400} TESTS="tests/test_gemm_wgrad_gpu.py tests/test_update_gpu.py" PYARGS="-x -k wgrad" bash scripts/gpu_tests.sh || exit 1
for r in 16384 131072; do ROWS=$r SHAPE=wgrad timeout -k 10 120 python -u scripts/gemm_bench.py 2>/dev/null || exit 1; done
for it in 1 2; do
  timeout -k 10 200 python -u scripts/update_time.py --reps 5 2>/dev/null || exit 1
  timeout -k 10 200 python -u scripts/update_time.py --reps 5 --env LidarBicycleTarget --envs 512 --batch 2048 2>/dev/null || exit 1
done

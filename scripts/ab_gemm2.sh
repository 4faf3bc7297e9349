#!/bin/bash
# GEMM rows-path shapes after the epilogue-operand change, the GEMM / net / update parity tests, and the update
# time at the bench config (3 iterations of collect + update).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
SHAPE=fwd timeout -k 10 120 python scripts/gemm_bench.py || exit 1
SHAPE=dx timeout -k 10 120 python scripts/gemm_bench.py || exit 1
timeout -k 10 300 python -u -m pytest tests/test_nets_gpu.py tests/test_update_gpu.py tests/test_update_dynamics_gpu.py -x -q -m gpu --timeout 180 --timeout-method thread -p no:cacheprovider 2>&1 | tail -3
ENV_ID=LidarSpread N_AGENTS=8 N_OBS=3 N_ENV=4096 T=128 BATCH=16384 ITERS=4 MARK_UPDATE=0 timeout -k 10 300 python scripts/update_smoke.py 2>&1 | grep iter

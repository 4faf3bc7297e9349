#!/bin/bash
# A/B of the whole-unit prefetch rows kernel (DGPPO_ROWS_PF) on the update's GEMM shapes, plus its parity tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
COPY=1 SHAPE=none timeout -k 10 120 python scripts/gemm_bench.py || exit 1
for pf in 0 1; do for wg in 0 2 3; do
  echo "== PF $pf WG/CU $wg"
  DGPPO_ROWS_PF=$pf DGPPO_ROWS_WG_PER_CU=$wg SHAPE=fwd timeout -k 10 120 python scripts/gemm_bench.py || exit 1
  DGPPO_ROWS_PF=$pf DGPPO_ROWS_WG_PER_CU=$wg SHAPE="dx N64 K64" timeout -k 10 120 python scripts/gemm_bench.py || exit 1
done; done
DGPPO_ROWS_PF=1 timeout -k 10 300 python -u -m pytest tests/test_nets_gpu.py tests/test_update_gpu.py -x -q -m gpu --timeout 180 --timeout-method thread -p no:cacheprovider 2>&1 | tail -3

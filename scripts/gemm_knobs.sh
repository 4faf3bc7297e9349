#!/bin/bash
# A/B of the GEMM launch knobs on the update's dominant shapes (scripts/gemm_bench.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for k in 0 1 2 3; do echo "== rows WG/CU $k"; DGPPO_ROWS_WG_PER_CU=$k SHAPE=fwd timeout -k 10 120 python scripts/gemm_bench.py || exit 1; done
for k in 0 1 2; do echo "== rows dx WG/CU $k"; DGPPO_ROWS_WG_PER_CU=$k SHAPE=dx timeout -k 10 120 python scripts/gemm_bench.py || exit 1; done
for mr in 512 128 64; do for ma in 12 6 4; do echo "== wgrad minrows $mr maxacc $ma"; DGPPO_WGRAD_MINROWS=$mr DGPPO_WGRAD_MAXACC=$ma SHAPE=wgrad timeout -k 10 120 python scripts/gemm_bench.py || exit 1; done; done
echo "== wgrad small K"; for mr in 512 128 64; do DGPPO_WGRAD_MINROWS=$mr ROWS=16384 SHAPE=wgrad timeout -k 10 120 python scripts/gemm_bench.py || exit 1; done

#!/bin/bash
# A/B of rows-GEMM launch variants on the dominant shapes (scripts/gemm_bench.py); VARS="KNOB=v ..." lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 200 python -u -m pytest tests/test_nets_gpu.py -q -m gpu -k "gemm" -x --timeout 120 2>&1 | tail -1 || exit 1
while IFS= read -r v; do
  [ -z "$v" ] && continue
  echo "== $v"; env $v SHAPE="${SHAPE:-}" timeout -k 10 120 python scripts/gemm_bench.py 2>&1 | grep -v amdgpu.ids || exit 1
done <<< "${VARS:-DGPPO_ROWS_NTW=0}"

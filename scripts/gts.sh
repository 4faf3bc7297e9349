#!/bin/bash
# Per-shape GEMM time of one DGPPO update (scripts/gemm_time_by_shape.py) under rocprofv3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gts -o upd -- \
  python3 scripts/gemm_time_by_shape.py gpurun_out/gemm_log.json > gpurun_out/gts.log 2>&1 || { tail -20 gpurun_out/gts.log; exit 1; }
python3 scripts/gemm_time_by_shape.py --analyze gpurun_out/gts/upd_kernel_trace.csv gpurun_out/gemm_log.json
python3 scripts/top_kernels.py gpurun_out/gts/upd_kernel_stats.csv 30 2>/dev/null || true

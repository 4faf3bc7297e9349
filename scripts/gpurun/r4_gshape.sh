#!/bin/bash
# round 4: per-shape GEMM time of one update (serial streams so kernels match their calls)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/gshape
export TMPDIR=/tmp DGPPO_STREAMS=0
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gshape -o upd -- python3 scripts/gemm_time_by_shape.py gpurun_out/gshape/gemm_log.json > gpurun_out/gshape/run.log 2>&1 || exit $?
f=$(ls gpurun_out/gshape/*kernel_trace.csv gpurun_out/gshape/*/*kernel_trace.csv 2>/dev/null | head -n 1)
echo "trace $f"
python3 scripts/gemm_time_by_shape.py --analyze "$f" gpurun_out/gshape/gemm_log.json > gpurun_out/gshape/shapes.txt 2>&1
head -n 40 gpurun_out/gshape/shapes.txt
rm -f gpurun_out/gshape/*kernel_trace.csv gpurun_out/gshape/*/*kernel_trace.csv

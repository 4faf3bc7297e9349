#!/bin/bash
# kernel times of one minibatch's passes, graph-form MFMA vs row-block attention (scripts/attn_gm_ab.py), and a PMC
# pass over the gm kernels
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/gmprof
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/gmprof/trace -o run --output-format csv -- python3 scripts/attn_gm_ab.py > gpurun_out/gmprof/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
f=$(ls gpurun_out/gmprof/trace/*/run_kernel_stats.csv 2>/dev/null || find gpurun_out/gmprof/trace -name "*kernel_stats.csv" | head -1)
head -30 $f | cut -c1-200
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_F32 --kernel-include-regex attn_ -d gpurun_out/gmprof/pmc -o run --output-format csv -- python3 scripts/attn_gm_ab.py > gpurun_out/gmprof/pmc.log 2>&1
echo "pmc rc=$?"
exit 0

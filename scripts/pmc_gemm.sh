#!/bin/bash
# PMC passes for one GEMM shape of scripts/gemm_bench.py (SHAPE substring, ITERS launches): one counter group per
# rocprofv3 run, kernel-trace only.  Usage: SHAPE="wgrad M64 N64" bash scripts/pmc_gemm.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pmcg
mkdir -p $OUT
export TMPDIR=/tmp ITERS=${ITERS:-10}
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
           "FETCH_SIZE" "WRITE_SIZE" \
           "GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SMEM SQ_INST_LEVEL_VMEM" \
           "TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_LATENCY_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex "${KRE:-gemm}" -d $OUT/p$i -o run \
    --output-format csv -- python3 scripts/gemm_bench.py > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/p$i.log; exit $rc; }
done
python3 scripts/pmc_table.py $OUT

#!/bin/bash
# PMC passes over scripts/gemm_bench.py (one shape) + the HBM copy calibration.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/gpmc; mkdir -p $OUT; export TMPDIR=/tmp
COPY=1 SHAPE=NONE timeout -k 10 60 python scripts/gemm_bench.py 2>&1 | grep copy
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
           "FETCH_SIZE" "WRITE_SIZE" \
           "GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU_MFMA_MOPS_F32"; do
  i=$((i+1))
  ITERS=3 SHAPE="${SHAPE:-fwd N64 K64 +b}" timeout -k 10 60 rocprofv3 --kernel-trace --pmc $grp -d $OUT/p$i -o run --output-format csv -- python3 scripts/gemm_bench.py > $OUT/p$i.log 2>&1
  echo "pass $i rc=$?"
done
python3 scripts/pmc_table.py $OUT

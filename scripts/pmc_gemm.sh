#!/bin/bash
# PMC passes for the GEMM kernels on one gemm_bench shape: SHAPE='N64 K64 +b' bash scripts/pmc_gemm.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pmcg
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS" \
           "GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_VMEM SQ_WAIT_INST_ANY" ; do
  i=$((i+1))
  ITERS=3 timeout -k 10 200 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex "${KRE:-gemm_}" \
      -d $OUT/p$i -o run --output-format csv -- python3 scripts/gemm_bench.py > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  if fatal $rc; then exit $rc; fi
done
python3 scripts/pmc_table.py $OUT

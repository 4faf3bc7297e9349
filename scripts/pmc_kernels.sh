#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only) for kernels matching $KRE
# while running DGPPO collect+update (1 iteration).  Usage: KRE='attn_' bash scripts/pmc_kernels.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pmck
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
i=0
GROUPS_DEFAULT=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
  "FETCH_SIZE" "WRITE_SIZE"
  "GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS")
if [ -n "$PMC_GROUPS" ]; then IFS='|' read -r -a GROUPS_RUN <<< "$PMC_GROUPS"; else GROUPS_RUN=("${GROUPS_DEFAULT[@]}"); fi
for grp in "${GROUPS_RUN[@]}"; do
  i=$((i+1))
  ENV_ID=LidarSpread N_AGENTS=8 N_OBS=3 N_ENV=${N_ENV:-4096} T=128 BATCH=16384 ITERS=1 \
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex "${KRE:-attn_}" \
      -d $OUT/p$i -o run --output-format csv -- python3 scripts/update_smoke.py > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  if fatal $rc; then exit $rc; fi
done
python3 scripts/pmc_table.py $OUT

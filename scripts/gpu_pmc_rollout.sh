#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only) for the persistent env rollout
# kernel, plus a plain kernel-trace --stats run of the same driver.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pmcr
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 scripts/rollout_only.py > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; if fatal $rc; then exit $rc; fi
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
           "GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_TRANS_F32"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex rollout -d $OUT/p$i -o run \
      --output-format csv -- python3 scripts/rollout_only.py > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"
  if fatal $rc; then exit $rc; fi
done
python3 scripts/pmc_summary.py $OUT lidar_rollout_wave_kernel gpurun_out/env_rollout_pmc.json > /dev/null && echo summarised
exit 0

#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel-trace only) for the env-step kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
           "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_TRANS_F32" ; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --kernel-trace --pmc $grp -d gpurun_out/pmc/p$i -o run --output-format csv -- \
      python3 scripts/step_only.py > gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pass $i ($grp) rc=$rc"
  if fatal $rc; then exit $rc; fi
done
exit 0

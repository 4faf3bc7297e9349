#!/bin/bash
# PMC passes on the env-step kernels (scripts/env_dbg.py: full, graph-only, compute-only variants).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pmce
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
           "GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex "${KRE:-wave}" \
      -d $OUT/p$i -o run --output-format csv -- python3 ${SCRIPT:-scripts/step_only.py} > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  if fatal $rc; then exit $rc; fi
done
exit 0

#!/bin/bash
# MFMA utilisation of the update's kernels from PMC counters: one rocprofv3 --pmc pass (executed fp32 MFMA
# ops, MFMA busy cycles) and one plain kernel-trace pass (durations) over one DGPPO collect + update at the
# bench config; scripts/mfma_util.py joins them per kernel family.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/mfma
mkdir -p $OUT
export TMPDIR=/tmp ENV_ID=LidarSpread N_AGENTS=8 N_OBS=3 N_ENV=4096 T=128 BATCH=16384 ITERS=3
# executed fp32 work: MFMA ops and (round 5) the VALU's fp32 flops, with a calibration run of known elementwise work
PMC="SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_FLOPS_FP32_TRANS GRBM_GUI_ACTIVE"
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $PMC -d $OUT/calib -o run --output-format csv -- \
  python3 scripts/valu_calib.py > $OUT/calib.log 2>&1
rc=$?; echo "calib rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $PMC \
  -d $OUT/pmc -o run --output-format csv -- python3 scripts/update_smoke.py > $OUT/pmc.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 240 rocprofv3 --kernel-trace -d $OUT/trace -o run --output-format csv -- \
  python3 scripts/update_smoke.py > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 scripts/mfma_util.py $OUT

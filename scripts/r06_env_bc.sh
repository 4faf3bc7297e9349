#!/bin/bash
# round 6 diagnostic: SQ_LDS_BANK_CONFLICT of the env rollout with one LDS phase dropped per build (DGPPO_DIAG_BC=k,
# results invalid; attribution only): prev = the shipped source, bc1 no cast atomics, bc2 no rank loop, bc3 no F2
# staging writes, bc4 no ray cast
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
grp="GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU"
for lib in ${LIBS:-prev bc1 bc2 bc3 bc4}; do
  export DGPPO_HIP_LIB=$PWD/dgppo_fov_amd/lib/libdgppo_hip_$lib.so
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex rollout -d gpurun_out/bc_$lib/p1 -o run \
      --output-format csv -- python3 scripts/rollout_only.py > gpurun_out/bc_$lib.log 2>&1 || exit 1
  echo $lib; python3 scripts/pmc_summary.py gpurun_out/bc_$lib lidar_rollout_wave_kernel gpurun_out/bc_$lib.json | grep -A6 avg_per
done

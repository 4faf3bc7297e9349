#!/bin/bash
# round 6: env rollout LDS change: env / rollout parity tests, interleaved episode A/B against libdgppo_hip_prev.so,
# then the bank-conflict PMC group on the in-tree library (and the previous one)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TLIM=400 TESTS="tests/test_env_gpu.py tests/test_rollout_gpu.py" bash scripts/gpu_tests.sh | tail -3 || exit 1
rm -f gpurun_out/ab_new.txt gpurun_out/ab_prev.txt
bash scripts/ab_env.sh || exit 1
echo new; cat gpurun_out/ab_new.txt; echo prev; cat gpurun_out/ab_prev.txt
export TMPDIR=/tmp
grp="GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU"
for lib in new prev; do
  if [ $lib = prev ]; then export DGPPO_HIP_LIB=$PWD/dgppo_fov_amd/lib/libdgppo_hip_prev.so; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex rollout -d gpurun_out/bc_$lib/p1 -o run \
      --output-format csv -- python3 scripts/rollout_only.py > gpurun_out/bc_$lib.log 2>&1 || exit 1
  python3 scripts/pmc_summary.py gpurun_out/bc_$lib lidar_rollout_wave_kernel gpurun_out/bc_$lib.json | grep -A8 avg_per
done

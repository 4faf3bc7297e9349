#!/bin/bash
# graph-form agent-mode backward (n = 32): parity, per-pass kernel split vs the block kernel; trajectory-test A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PT="python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 $PT tests/test_nets_gpu.py tests/test_update_gpu.py -k "32" > gpurun_out/g32_tests.log 2>&1
rc=$?; echo "n32 tests rc=$rc"; tail -5 gpurun_out/g32_tests.log; grep -h 'Error' gpurun_out/g32_tests.log | head -5; [ $rc -eq 0 ] || exit $rc
T=tests/test_update_dynamics_gpu.py::test_trajectory_matches_oracle_loop
for kn in "DGPPO_ATTN_FWD2=lds" "DGPPO_ROWS_PF=0" "DGPPO_ROWS_BREG=0" "DGPPO_ATTN_FWD2=lds DGPPO_ATTN_BWD2=lds"; do
  env $kn timeout -k 10 200 $PT -x "$T" > gpurun_out/traj_ab.log 2>&1; echo "$kn rc=$?"; grep -h 'AssertionError:' gpurun_out/traj_ab.log | head -2
done
for v in 1 0; do
  DGPPO_ATTN_GBWD32=$v MB_N=32 MB_OBS=8 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/mb32_$v -o mb -- \
    python3 scripts/mb_profile.py > gpurun_out/mb32_$v.log 2>&1 || { echo "mb_profile failed"; tail -20 gpurun_out/mb32_$v.log; exit 1; }
  python3 scripts/mb_profile.py --split gpurun_out/mb32_$v/mb_kernel_trace.csv > gpurun_out/mb32_split_$v.txt && cat gpurun_out/mb32_split_$v.txt | grep -E '==|attn'
done
for v in 1 0; do DGPPO_WGRAD_NT4=$v ITERS=50 timeout -k 10 120 python3 scripts/gemm_bench.py 2>&1 | grep -E 'wgrad' | sed "s/^/nt4=$v /"; done

#!/bin/bash
# round 6: update-kernel change: nets / layer / update / trajectory parity tests, interleaved update A/B of the in-tree
# library against libdgppo_hip_$PREV.so (bench config and config 4's share), attention kernel stats under rocprof
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
PREV=${PREV:-aprev}
TLIM=600 TESTS="${UTESTS:-tests/test_update_gpu.py tests/test_gnn_layer_gpu.py tests/test_nets_gpu.py tests/test_update_dynamics_gpu.py}" bash scripts/gpu_tests.sh | tail -4 || exit 1
for it in 1 2; do
  for lib in main $PREV; do
    L=$PWD/dgppo_fov_amd/lib/libdgppo_hip.so; [ $lib = main ] || L=$PWD/dgppo_fov_amd/lib/libdgppo_hip_$lib.so
    echo "$lib $(DGPPO_HIP_LIB=$L timeout -k 10 200 python -u scripts/update_time.py --reps 5 2>/dev/null | tail -1)" || exit 1
    echo "$lib c4 $(DGPPO_HIP_LIB=$L timeout -k 10 200 python -u scripts/update_time.py --reps 5 --env LidarBicycleTarget --envs 512 --batch 2048 2>/dev/null | tail -1)" || exit 1
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/uab -o run --output-format csv -- \
  python3 scripts/update_time.py --reps 1 > gpurun_out/uab.log 2>&1 || { tail gpurun_out/uab.log; exit 1; }
python3 scripts/top_kernels.py gpurun_out/uab/run_kernel_stats.csv 14
rm -f gpurun_out/uab/run_kernel_trace.csv

#!/bin/bash
# round 6 diagnostic: attention backward time attribution (DGPPO_DIAG_BWD builds, results invalid): per build the
# update under rocprofv3 --kernel-trace --stats and the attn_bwd2r rows of its kernel stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
libpath() { [ $1 = main ] && echo $PWD/dgppo_fov_amd/lib/libdgppo_hip.so || echo $PWD/dgppo_fov_amd/lib/libdgppo_hip_$1.so; }
for lib in ${ALIBS:-main d1 d2 d4}; do
  DGPPO_HIP_LIB=$(libpath $lib) timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ad_$lib -o run --output-format csv -- \
    python3 scripts/update_time.py --reps 1 > gpurun_out/ad_$lib.log 2>&1 || { tail gpurun_out/ad_$lib.log; exit 1; }
  echo "== $lib"; python3 scripts/top_kernels.py gpurun_out/ad_$lib/run_kernel_stats.csv 40 | grep -E "total|attn_bwd2r|gnn_layer_fwd|wgrad_grouped"
  rm -f gpurun_out/ad_$lib/run_kernel_trace.csv
done

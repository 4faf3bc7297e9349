#!/bin/bash
# round 6: fused policy step per-call time (scripts/policy_time.py, HIP events) for the in-tree library and the builds
# named in PLIBS (dgppo_fov_amd/lib/libdgppo_hip_X.so), interleaved, 3 rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2 3; do
  for lib in main ${PLIBS:-pd1}; do
    L=$PWD/dgppo_fov_amd/lib/libdgppo_hip.so; [ $lib = main ] || L=$PWD/dgppo_fov_amd/lib/libdgppo_hip_$lib.so
    echo "$lib $(DGPPO_HIP_LIB=$L timeout -k 10 120 python -u scripts/policy_time.py 4096 2>/dev/null | tail -1)" || exit 1
  done
done

#!/bin/bash
# kernel stats of the bench-config update with the fused epilogues on / off
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/fuseprof
export TMPDIR=/tmp
for k in 1 0; do
  DGPPO_FUSE_LN=$k timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/fuseprof/f$k -o run --output-format csv -- python3 scripts/update_time.py --reps 2 > gpurun_out/fuseprof/f$k.log 2>&1
  rc=$?; echo "fuse=$k rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0

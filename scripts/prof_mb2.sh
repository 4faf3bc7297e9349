#!/bin/bash
# Per-pass kernel split of one DGPPO minibatch (scripts/mb_profile.py) under rocprofv3, for the knob settings in
# $KNOBS (space-separated NAME=VALUE lists separated by commas), e.g. KNOBS="DGPPO_FUSED_LAYER=1,DGPPO_FUSED_LAYER=0".
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
IFS=',' read -ra SETS <<< "${KNOBS:-DGPPO_FUSED_LAYER=1}"
i=0
for s in "${SETS[@]}"; do
  i=$((i+1))
  env $s timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/mb$i -o mb -- \
    python3 scripts/mb_profile.py > gpurun_out/mb$i.log 2>&1 || { echo "mb_profile failed ($s)"; tail -20 gpurun_out/mb$i.log; exit 1; }
  echo "=== $s"
  python3 scripts/mb_profile.py --split gpurun_out/mb$i/mb_kernel_trace.csv > gpurun_out/mb_split$i.txt && cat gpurun_out/mb_split$i.txt
done

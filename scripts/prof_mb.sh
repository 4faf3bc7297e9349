#!/bin/bash
# Per-pass kernel split of one DGPPO minibatch (scripts/mb_profile.py) + whole collect+update stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/mb -o mb -- \
  python3 scripts/mb_profile.py > gpurun_out/mb.log 2>&1 || { echo "mb_profile failed"; tail -20 gpurun_out/mb.log; exit 1; }
cat gpurun_out/mb.log
python3 scripts/mb_profile.py --split gpurun_out/mb/mb_kernel_trace.csv > gpurun_out/mb_split.txt && cat gpurun_out/mb_split.txt

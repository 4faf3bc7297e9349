#!/bin/bash
# GPU idle inside one update, eager vs minibatch hipGraph replay (DGPPO_UPDATE_GRAPH), from kernel traces.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for g in 0 1; do
  DGPPO_UPDATE_GRAPH=$g timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gaps$g -o run -- \
    python3 scripts/update_time.py --reps 1 > gpurun_out/gaps$g.log 2>&1 || { tail gpurun_out/gaps$g.log; exit 1; }
  echo "== DGPPO_UPDATE_GRAPH=$g"; python3 scripts/mb_gaps.py gpurun_out/gaps$g || exit 1
done

#!/bin/bash
# Kernel statistics of DGPPO updates at the bench config (scripts/update_time.py under rocprofv3 --kernel-trace
# --stats) plus the live update time with the phase split; $KN adds knobs (e.g. KN="DGPPO_FUSED_LAYER=0").
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/up
export TMPDIR=/tmp
env $KN DGPPO_PHASE_EVENTS=1 timeout -k 10 300 python3 scripts/update_time.py --reps 5 > gpurun_out/up/live.json 2>gpurun_out/up/live.err || exit 1
cat gpurun_out/up/live.json
env $KN timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/up/prof -o up -- \
  python3 scripts/update_time.py --reps 1 > gpurun_out/up/prof.log 2>&1 || { tail -20 gpurun_out/up/prof.log; exit 1; }
python3 scripts/top_kernels.py $(ls gpurun_out/up/prof/*kernel_stats.csv gpurun_out/up/prof/*/*kernel_stats.csv 2>/dev/null | head -1) 45 > gpurun_out/up/top.txt 2>&1; cat gpurun_out/up/top.txt

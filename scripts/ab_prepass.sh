#!/bin/bash
# A/B of the update's prepass chunk size (DGPPO_PREPASS_GRAPHS) at the bench config: 3 collect + update iterations.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for g in 65536 262144 65536 262144; do
  DGPPO_PREPASS_GRAPHS=$g ENV_ID=LidarSpread N_AGENTS=8 N_OBS=3 N_ENV=4096 T=128 BATCH=16384 ITERS=4 \
    timeout -k 10 200 python3 scripts/update_smoke.py 2>&1 | grep -E "^iter [23]" | sed "s/^/graphs $g: /" || exit 1
done

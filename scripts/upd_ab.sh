#!/bin/bash
# Update wall time at the bench config with / without the concurrent-stream passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for st in ${STREAMS_AB:-0 1}; do
  echo "== DGPPO_STREAMS=$st"
  DGPPO_STREAMS=$st ENV_ID=LidarSpread N_AGENTS=8 N_OBS=3 N_ENV=4096 T=128 BATCH=16384 ITERS=${ITERS:-3} \
    timeout -k 10 300 python scripts/update_smoke.py 2>&1 | grep -E "^iter" || exit 1
done

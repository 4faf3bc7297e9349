#!/bin/bash
# Minibatch hipGraph replay at the bench config (16,384-sample minibatches): DGPPO_UPDATE_GRAPH=1 vs 0, interleaved,
# with the device-event phase split (DGPPO_PHASE_EVENTS=1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for i in 1 2; do
  for g in 1 0; do
    DGPPO_PHASE_EVENTS=1 DGPPO_UPDATE_GRAPH=$g timeout -k 10 300 python3 scripts/update_time.py --reps 5 2>/dev/null | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('graph=$g', d['collect_ms'], d['update_ms'], d['update_ms_all'], d['phases_ms'])" || exit 1
  done
done

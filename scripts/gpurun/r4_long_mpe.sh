#!/bin/bash
# round 4: the quickstart learning runs on MPESpread (BASELINE config 2's env), DGPPO and InforMARL side by side,
# resumed across calls (scripts/long_run.sh with ENV=MPESpread)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ENV=MPESpread RUNS="dgppo:0 informarl:0" MIN=16 bash scripts/long_run.sh

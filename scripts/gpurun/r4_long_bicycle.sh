#!/bin/bash
# round 4: the quickstart learning runs on LidarBicycleTarget (BASELINE config 4's env), DGPPO and InforMARL side by side,
# resumed across calls (scripts/long_run.sh with ENV=LidarBicycleTarget)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ENV=LidarBicycleTarget RUNS="dgppo:0 informarl:0" MIN=16 bash scripts/long_run.sh

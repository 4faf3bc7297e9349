#!/bin/bash
# round 4: two more DGPPO seeds of the LidarBicycleTarget quickstart (fresh; scripts/long_run.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ENV=LidarBicycleTarget RUNS="dgppo:1 dgppo:2" MIN=16 bash scripts/long_run.sh

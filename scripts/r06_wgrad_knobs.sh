#!/bin/bash
# round 6: the grouped weight-gradient kernel's chunking / in-flight knobs at the bench config and config 4's share
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for kn in "X=0" "DGPPO_WGRAD_MAXCHUNKS=512" "DGPPO_WGRAD_MAXCHUNKS=1024" "DGPPO_WGRAD_U=8" "DGPPO_WGRAD_U=8 DGPPO_WGRAD_MAXCHUNKS=512" "X=0"; do
  echo "$kn $(env $kn timeout -k 10 200 python -u scripts/update_time.py --reps 4 2>/dev/null | tail -1 | cut -c1-110)" || exit 1
  echo "$kn c4 $(env $kn timeout -k 10 200 python -u scripts/update_time.py --reps 4 --env LidarBicycleTarget --envs 512 --batch 2048 2>/dev/null | tail -1 | cut -c1-120)" || exit 1
done

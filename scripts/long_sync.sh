#!/bin/bash
# Between gpurun calls of scripts/long_run.sh: make the runs the last call left in gpurun_out/long/
# the ones the next call resumes (runs_long/ travels to the GPU box with the snapshot; it is git-ignored).
cd "$(dirname "$0")/.."
ENV=${ENV:-LidarSpread}
[ -d gpurun_out/long/$ENV ] || { echo "nothing to sync"; exit 1; }
mkdir -p runs_long && rm -rf runs_long/$ENV
cp -r gpurun_out/long/$ENV runs_long/
du -sh runs_long

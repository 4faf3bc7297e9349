#!/bin/bash
# config 4 (LidarBicycleTarget n8 o3, 4096 envs over 8 GPUs): the per-GPU weak share (4096 envs) and the strong
# share (512 envs, 2048-sample rank minibatch) with the env kernel choices and the minibatch hipGraph replay
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
O=gpurun_out/cfg4.jsonl
: > $O
run() { timeout -k 10 300 "$@" >> $O 2>> gpurun_out/cfg4.err; rc=$?; echo "rc=$rc: $*"; case $rc in 0) ;; *) exit $rc;; esac; }
run python -u scripts/config_bench.py --only "Bicycle" --reps 3
run python -u scripts/config_bench.py --only "x512" --reps 3 --step-kernel block
DGPPO_UPDATE_GRAPH=1 run python -u scripts/config_bench.py --only "x512" --reps 3
DGPPO_UPDATE_GRAPH=1 run python -u scripts/config_bench.py --only "x512" --reps 3 --step-kernel block
cat $O

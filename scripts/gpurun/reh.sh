#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
DGPPO_DIST_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --steps 5 --warmup 2 --ppo-iters 2 --no-cpu-baseline > gpurun_out/reh_weak.json 2> gpurun_out/reh_weak.err; rc=$?; echo "weak rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/reh_weak.err; exit $rc; }
cut -c1-400 gpurun_out/reh_weak.json
DGPPO_DIST_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --strong --steps 5 --warmup 2 --ppo-iters 2 --no-cpu-baseline > gpurun_out/reh_strong.json 2> gpurun_out/reh_strong.err; rc=$?; echo "strong rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/reh_strong.err; exit $rc; }
cut -c1-400 gpurun_out/reh_strong.json

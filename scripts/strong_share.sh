#!/bin/bash
# BASELINE configs 4 and 5 at their 8-GPU per-rank shares on one GPU (scripts/update_time.py):
#   config 4 strong: LidarBicycleTarget n8 o3, 4096 envs / 8 = 512 per rank, 16,384-sample minibatch / 8 = 2048;
#                    and the 4096-env single-GPU baseline the projection divides by
#   config 5:        LidarSpread n32 o8, 8192 envs / 8 = 1024 per rank, minibatch_plan at world 8 = 64 x 2048 samples
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out/${OUT:-strong.jsonl}
rm -f $OUT
for args in "--env LidarBicycleTarget --envs 4096 --batch 16384" "--env LidarBicycleTarget --envs 512 --batch 2048" \
            "--env LidarSpread -n 32 --obs 8 --envs 1024 --batch 2048"; do
  env $KN DGPPO_PHASE_EVENTS=1 timeout -k 10 400 python3 scripts/update_time.py $args --reps 5 >> $OUT 2>gpurun_out/strong.err || { tail gpurun_out/strong.err; exit 1; }
  tail -1 $OUT
done

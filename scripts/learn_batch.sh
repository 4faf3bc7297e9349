#!/bin/bash
# DGPPO learning runs on small configs (scripts/learning_run.py through train.py / test.py), each under its
# own time limit; results in gpurun_out/learn_<name>/learning_run.json.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
run() {  # name, then learning_run.py args
  local name=$1; shift
  timeout -k 10 300 python -u scripts/learning_run.py --out gpurun_out/learn_$name "$@" > gpurun_out/learn_$name.log 2>&1
  echo "$name rc=$?"
}
run mpet2 --env MPETarget -n 2 --obs 0 --algo dgppo --steps 300 --eval-interval 50 --epi 64 || exit 1
run lidt2_r128 --env LidarTarget -n 2 --obs 0 --algo dgppo --steps 300 --eval-interval 50 --epi 64 --rnn-step 128 || exit 1
run lids3_r128 --env LidarSpread -n 3 --obs 2 --algo dgppo --steps 500 --eval-interval 100 --epi 64 --rnn-step 128 || exit 1
run mpes3 --env MPESpread -n 3 --obs 3 --algo dgppo --steps 500 --eval-interval 100 --epi 64 || exit 1

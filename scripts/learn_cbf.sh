#!/bin/bash
# DGPPO on MPETarget n=2 (300 steps) with the CBF advantage weight at 0 / 0.1 / the default 1 (cbf schedule on):
# does the CBF term drive the early collapse?  Results in gpurun_out/learn_cbf<w>/learning_run.json.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for w in 0 0.1 1; do
  timeout -k 10 300 python -u scripts/learning_run.py --out gpurun_out/learn_cbf$w --env MPETarget -n 2 --obs 0 \
    --algo dgppo --steps 300 --eval-interval 50 --epi 64 --cbf-weight $w > gpurun_out/learn_cbf$w.log 2>&1
  echo "cbf $w rc=$?"
done

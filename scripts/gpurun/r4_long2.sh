#!/bin/bash
# round 4: second long-run segment (DGPPO seed 0 resumed, seeds 1 and 2 from scratch) with the GPU test suite
# running beside it (the runs use a fraction of the GPU at 128 envs)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
RUNS="dgppo:0 dgppo:1 dgppo:2" MIN=16 bash scripts/long_run.sh > gpurun_out/long_run_driver.log 2>&1 &
lp=$!
sleep 20
TLIM=600 bash scripts/gpu_tests.sh
trc=$?
echo "tests rc=$trc"
wait $lp
lrc=$?
echo "long rc=$lrc"
tail -n 5 gpurun_out/long_run_driver.log
exit $(( trc != 0 ? trc : lrc ))

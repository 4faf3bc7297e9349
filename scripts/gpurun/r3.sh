#!/bin/bash
# round-3 re-entry check: the trajectory test under both attention-backward forms, the default bench line, then
# this round's profiles
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
T=tests/test_update_dynamics_gpu.py::test_trajectory_matches_oracle_loop
timeout -k 10 300 python -u -m pytest "$T" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_traj_reg.log 2>&1; echo "reg rc=$?"
DGPPO_ATTN_BWD2=lds timeout -k 10 300 python -u -m pytest "$T" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_traj_lds.log 2>&1; echo "lds rc=$?"
grep -h 'AssertionError' gpurun_out/r3_traj_*.log
timeout -k 10 400 python3 bench.py > gpurun_out/r3_bench.json 2> gpurun_out/r3_bench.err || { tail -20 gpurun_out/r3_bench.err; exit 1; }
cat gpurun_out/r3_bench.json | cut -c1-600
bash scripts/round_profiles.sh > gpurun_out/r3_round_profiles.txt 2>&1; rc=$?; tail -40 gpurun_out/r3_round_profiles.txt; exit $rc

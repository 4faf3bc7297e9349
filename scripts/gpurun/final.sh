#!/bin/bash
# this round's evidence on the current build: GPU parity suite, the default bench line, bench kernel stats +
# executed-MFMA PMC + env-rollout PMC (scripts/round_profiles.sh), every BASELINE config (scripts/config_bench.py)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
TLIM=600 PYARGS=" " bash scripts/gpu_tests.sh > gpurun_out/final_tests_tail.txt 2>&1; rc=$?
grep -E 'passed|failed' gpurun_out/pytest_gpu.log | tail -2; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err || { tail -20 gpurun_out/final_bench.err; exit 1; }
cut -c1-300 gpurun_out/final_bench.json
bash scripts/round_profiles.sh > gpurun_out/final_round_profiles.txt 2>&1 || { tail -30 gpurun_out/final_round_profiles.txt; exit 1; }
tail -5 gpurun_out/final_round_profiles.txt
timeout -k 10 900 python3 scripts/config_bench.py > gpurun_out/final_config_bench.jsonl 2> gpurun_out/final_config_bench.err || { tail -5 gpurun_out/final_config_bench.err; exit 1; }
grep -c config gpurun_out/final_config_bench.jsonl

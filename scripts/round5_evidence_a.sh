#!/bin/bash
# Round-5 evidence, part A, on the final tree: the GPU test suite, the bench line, the bench under rocprofv3 --stats,
# the executed-fp32 PMC passes (profiles/r05_mfma_util.json's source) and the env rollout PMC passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TLIM=600 bash scripts/gpu_tests.sh > gpurun_out/ev_tests_tail.txt 2>&1 || { tail -20 gpurun_out/ev_tests_tail.txt; exit 1; }
tail -2 gpurun_out/ev_tests_tail.txt
timeout -k 10 400 python3 bench.py > gpurun_out/r05_bench_final.json 2> gpurun_out/r05_bench_final.err || { tail gpurun_out/r05_bench_final.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r05_bench_final.json').read().strip().splitlines()[-1]);print(d['value'], d['roofline']['frac'], d['ppo']['update_ms'], d['ppo']['collect_ms'])"
bash scripts/round_profiles.sh > gpurun_out/ev_rp.txt 2>&1 || { tail -20 gpurun_out/ev_rp.txt; exit 1; }
tail -5 gpurun_out/ev_rp.txt

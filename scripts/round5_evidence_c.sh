#!/bin/bash
# Round-5 evidence, part C: every BASELINE config on one GPU (scripts/config_bench.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 1000 python3 -u scripts/config_bench.py > gpurun_out/r05_config_bench.jsonl 2> gpurun_out/config_bench.err || { tail gpurun_out/config_bench.err; exit 1; }
wc -l gpurun_out/r05_config_bench.jsonl

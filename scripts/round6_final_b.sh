#!/bin/bash
# Round-6 closing evidence, part B: update HBM traffic per kernel family (PMC), configs 4 / 5 per-rank shares, the
# kernel list of config 4's 2048-sample minibatches, every BASELINE config on one GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/update_traffic_pmc.sh > gpurun_out/ev_traffic.txt 2>&1 || { tail -20 gpurun_out/ev_traffic.txt; exit 1; }
tail -3 gpurun_out/ev_traffic.txt
OUT=r06_strong.jsonl bash scripts/strong_share.sh || exit 1
bash scripts/r06_c4_trace.sh > gpurun_out/r06_c4_trace_out.txt 2>&1 || { tail gpurun_out/r06_c4_trace_out.txt; exit 1; }
head -3 gpurun_out/c4_kernels.txt
timeout -k 10 1000 python3 -u scripts/config_bench.py > gpurun_out/r06_config_bench.jsonl 2> gpurun_out/config_bench.err || { tail gpurun_out/config_bench.err; exit 1; }
wc -l gpurun_out/r06_config_bench.jsonl

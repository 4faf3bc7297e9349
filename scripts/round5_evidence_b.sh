#!/bin/bash
# Round-5 evidence, part B: update HBM traffic per kernel family (PMC), configs 4 / 5 per-rank shares.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash scripts/update_traffic_pmc.sh > gpurun_out/ev_traffic.txt 2>&1 || { tail -20 gpurun_out/ev_traffic.txt; exit 1; }
tail -3 gpurun_out/ev_traffic.txt
OUT=r05_strong.jsonl bash scripts/strong_share.sh || exit 1

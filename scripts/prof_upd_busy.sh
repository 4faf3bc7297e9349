#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
ENV_ID=LidarSpread N_AGENTS=8 N_OBS=3 N_ENV=4096 T=128 BATCH=16384 ITERS=2 \
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pub -o upd --output-format csv -- \
  python3 scripts/update_smoke.py > gpurun_out/pub.log 2>&1 || { tail -5 gpurun_out/pub.log; exit 1; }
grep -E "^iter" gpurun_out/pub.log
python3 scripts/busy.py gpurun_out/pub/upd_kernel_trace.csv 20000000
python3 scripts/top_kernels.py gpurun_out/pub/upd_kernel_stats.csv 12

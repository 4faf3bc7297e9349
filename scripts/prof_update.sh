#!/bin/bash
# rocprofv3 kernel trace + stats of DGPPO collect+update at the bench config (2 iterations).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
ENV_ID=LidarSpread N_AGENTS=8 N_OBS=3 N_ENV=4096 T=128 BATCH=16384 ITERS=${ITERS:-2} \
  timeout -k 10 ${TLIM:-400} rocprofv3 --kernel-trace --stats -d gpurun_out/prof_upd -o upd --output-format csv -- \
  python3 scripts/update_smoke.py > gpurun_out/prof_upd.log 2>&1
rc=$?; echo "rocprof rc=$rc"; grep -E "^iter" gpurun_out/prof_upd.log
python3 scripts/top_kernels.py gpurun_out/prof_upd/upd_kernel_stats.csv 25
exit $rc

#!/bin/bash
# This round's committed evidence: rocprofv3 kernel stats of a short bench run, the executed-MFMA PMC pass of
# collect + update (scripts/mfma_pmc.sh) and the env rollout PMC passes (scripts/gpu_pmc_rollout.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/rp
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/rp/bench -o bench --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 --ppo-iters 3 --no-cpu-baseline > gpurun_out/rp/bench.log 2>&1
rc=$?; echo "bench under rocprof rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 scripts/top_kernels.py gpurun_out/rp/bench/bench_kernel_stats.csv 25
bash scripts/mfma_pmc.sh || exit 1
bash scripts/gpu_pmc_rollout.sh || exit 1

#!/bin/bash
# Round-6 closing evidence on the final tree, ordered so the bench line quotes this tree's profiles: the GPU test
# suite, the executed-fp32 PMC passes and the env rollout PMC passes (copied into profiles/ on the box before the
# bench reads them; copy gpurun_out/mfma/mfma_util.json and gpurun_out/env_rollout_pmc.json into profiles/ here
# afterwards), the bench line, then the bench under rocprofv3 --kernel-trace --stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TLIM=700 bash scripts/gpu_tests.sh > gpurun_out/fin_tests_tail.txt 2>&1 || { tail -20 gpurun_out/fin_tests_tail.txt; exit 1; }
tail -2 gpurun_out/fin_tests_tail.txt
bash scripts/mfma_pmc.sh > gpurun_out/fin_mfma.txt 2>&1 || { tail -20 gpurun_out/fin_mfma.txt; exit 1; }
cp gpurun_out/mfma/mfma_util.json profiles/r06_mfma_util.json
bash scripts/gpu_pmc_rollout.sh > gpurun_out/fin_pmcr.txt 2>&1 || { tail -20 gpurun_out/fin_pmcr.txt; exit 1; }
cp gpurun_out/env_rollout_pmc.json profiles/r06_env_rollout_pmc.json
timeout -k 10 400 python3 bench.py > gpurun_out/r06_bench_final.json 2> gpurun_out/r06_bench_final.err || { tail gpurun_out/r06_bench_final.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r06_bench_final.json').read().strip().splitlines()[-1]);print(d['value'], d['roofline']['frac'], d['ppo']['update_ms'], d['ppo']['collect_ms'], d['ppo']['update_roofline'].get('executed_mfma', {}).get('status', 'quoted'))"
export TMPDIR=/tmp
mkdir -p gpurun_out/rp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/rp/bench -o bench --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 --ppo-iters 3 --no-cpu-baseline > gpurun_out/rp/bench.log 2>&1
rc=$?; echo "bench under rocprof rc=$rc"; [ $rc -ne 0 ] && exit $rc
rm -f gpurun_out/rp/bench/bench_kernel_trace.csv
python3 scripts/top_kernels.py gpurun_out/rp/bench/bench_kernel_stats.csv 12

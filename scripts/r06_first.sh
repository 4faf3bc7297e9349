#!/bin/bash
# Round-6 first evidence on the restored tree: GPU test suite, bench line, bench under rocprofv3 --kernel-trace --stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TLIM=700 bash scripts/gpu_tests.sh > gpurun_out/r06_tests_tail.txt 2>&1 || { tail -30 gpurun_out/r06_tests_tail.txt; exit 1; }
tail -2 gpurun_out/r06_tests_tail.txt
timeout -k 10 400 python3 bench.py > gpurun_out/r06_bench.json 2> gpurun_out/r06_bench.err || { tail gpurun_out/r06_bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('gpurun_out/r06_bench.json').read().strip().splitlines()[-1]);print(d['value'], d['roofline']['frac'], d['ppo']['update_ms'], d['ppo']['collect_ms'])"
export TMPDIR=/tmp
mkdir -p gpurun_out/rp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/rp/bench -o bench --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 --ppo-iters 3 --no-cpu-baseline > gpurun_out/rp/bench.log 2>&1
rc=$?; echo "bench under rocprof rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 scripts/top_kernels.py gpurun_out/rp/bench/bench_kernel_stats.csv 16

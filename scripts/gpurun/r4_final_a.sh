#!/bin/bash
# round 4 final evidence (part A): GPU suite, smoke, bench line, bench kernel stats + executed-MFMA PMC + env
# rollout PMC (scripts/round_profiles.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/final
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/final/pytest_gpu.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -n 3 gpurun_out/final/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -n 2 gpurun_out/final/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
bash scripts/round_profiles.sh > gpurun_out/final/rp.log 2>&1
rc=$?; echo "round_profiles rc=$rc"; tail -n 4 gpurun_out/final/rp.log
exit $rc

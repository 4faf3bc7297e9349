#!/bin/bash
# round 4 evidence on the current build: bench line, bench kernel stats + executed-MFMA PMC + env-rollout PMC
# (scripts/round_profiles.sh), update HBM traffic PMC (scripts/update_traffic_pmc.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > gpurun_out/ev_bench.json 2> gpurun_out/ev_bench.err
rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/ev_bench.json; [ $rc -ne 0 ] && exit $rc
bash scripts/round_profiles.sh > gpurun_out/ev_rp.log 2>&1
rc=$?; echo "round_profiles rc=$rc"; tail -n 5 gpurun_out/ev_rp.log; [ $rc -ne 0 ] && exit $rc
bash scripts/update_traffic_pmc.sh > gpurun_out/ev_traffic.log 2>&1
rc=$?; echo "traffic rc=$rc"; tail -n 30 gpurun_out/ev_traffic.log
exit $rc

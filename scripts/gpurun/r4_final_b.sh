#!/bin/bash
# round 4 final evidence (part B): update HBM traffic PMC, every BASELINE config (scripts/config_bench.py), config 4's
# strong share with the live update phase split
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/final
export TMPDIR=/tmp
bash scripts/update_traffic_pmc.sh > gpurun_out/final/traffic.log 2>&1
rc=$?; echo "traffic rc=$rc"; tail -n 4 gpurun_out/final/traffic.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u scripts/config_bench.py > gpurun_out/final/config_bench.jsonl 2> gpurun_out/final/config_bench.err
rc=$?; echo "config_bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
: > gpurun_out/final/config4_strong.jsonl
for e in "--envs 4096 --batch 16384" "--envs 512 --batch 2048"; do
  DGPPO_PHASE_EVENTS=1 timeout -k 10 240 python -u scripts/update_time.py --env LidarBicycleTarget $e >> gpurun_out/final/config4_strong.jsonl 2>> gpurun_out/final/config4_strong.err || exit $?
done
cat gpurun_out/final/config4_strong.jsonl

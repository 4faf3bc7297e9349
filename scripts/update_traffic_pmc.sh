#!/bin/bash
# HBM traffic of one DGPPO update (the bench config) per kernel family: a FETCH_SIZE pass, a WRITE_SIZE pass
# (separate rocprofv3 --pmc runs, kernel-trace only) and a plain kernel trace over scripts/update_smoke.py;
# scripts/update_traffic.py keeps the dispatches after the last collect's `spin_kernel` marker (one update) and
# prices bytes as 2 x FETCH_SIZE + WRITE_SIZE (gfx950: FETCH_SIZE counts half the bytes of wide streaming reads).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/utraffic
mkdir -p $OUT
export TMPDIR=/tmp ENV_ID=LidarSpread N_AGENTS=8 N_OBS=3 N_ENV=4096 T=128 BATCH=16384 ITERS=2
fatal() { case "$1" in 0) return 1;; *) return 0;; esac; }
timeout -k 10 240 rocprofv3 --kernel-trace -d $OUT/trace -o run --output-format csv -- python3 scripts/update_smoke.py > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; if fatal $rc; then exit $rc; fi
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $c -d $OUT/$c -o run --output-format csv -- python3 scripts/update_smoke.py > $OUT/$c.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"; if fatal $rc; then exit $rc; fi
done
python3 scripts/update_traffic.py $OUT

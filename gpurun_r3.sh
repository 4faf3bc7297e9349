timeout -k 10 400 python -u -m pytest tests/test_rollout_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r3_tests.log; [ $rc -eq 0 ] || exit $rc
bash gpurun_mpeprof.sh > gpurun_out/mpeprof.txt 2>&1 || exit 1
f=$(find gpurun_out/mpe_prof -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 "$f" | head -4 | cut -c1-60,130-200
timeout -k 10 200 python -u scripts/config_bench.py --no-ppo --only "MPE" || exit 1

timeout -k 10 400 python -u -m pytest tests/test_rollout_gpu.py -x -q -m gpu --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/t8.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/t8.log
for o in "MPESpread" "n32" "LidarSpread n8"; do timeout -k 10 200 python -u scripts/config_bench.py --no-ppo --only "$o" || exit 1; done

cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
timeout -k 10 400 python -u -m pytest tests/test_rollout_gpu.py -x -q -m gpu --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/t8.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/t8.log; [ $rc -eq 0 ] || exit $rc
for o in "MPESpread" "n32" "LidarSpread n8"; do timeout -k 10 200 python -u scripts/config_bench.py --no-ppo --only "$o" || exit 1; done

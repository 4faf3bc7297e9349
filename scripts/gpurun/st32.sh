#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
PT="python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider"
timeout -k 10 300 $PT tests/test_env_gpu.py tests/test_rollout_gpu.py > gpurun_out/st32_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/st32_tests.log; grep -h 'Error' gpurun_out/st32_tests.log | head -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 scripts/block_stamps.py LidarSpread 32 8 1024 2>&1 | grep -E 'ticks'
timeout -k 10 200 python3 scripts/config_bench.py --no-ppo --only "n32 o8" 2>&1 | grep -v amdgpu.ids
DGPPO_ENV_STEP_KERNEL=block timeout -k 10 200 python3 scripts/config_bench.py --no-ppo --only "LidarSpread n8" 2>&1 | grep -v amdgpu.ids

#!/bin/bash
# round 6: interleaved LidarSpread n8 episode A/B over several env builds (LIBS: "main" = in-tree library, X =
# dgppo_fov_amd/lib/libdgppo_hip_X.so), the rollout parity tests on each variant, then the LDS PMC group per build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
LIBS=${LIBS:-main edge pad both}
libpath() { [ $1 = main ] && echo $PWD/dgppo_fov_amd/lib/libdgppo_hip.so || echo $PWD/dgppo_fov_amd/lib/libdgppo_hip_$1.so; }
for lib in $LIBS; do
  DGPPO_HIP_LIB=$(libpath $lib) timeout -k 10 300 python -u -m pytest tests/test_rollout_gpu.py tests/test_env_gpu.py -m gpu -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/abn_test_$lib.log 2>&1 || { echo "$lib tests failed"; tail -20 gpurun_out/abn_test_$lib.log; exit 1; }
  echo "$lib: $(tail -1 gpurun_out/abn_test_$lib.log)"
done
for i in 1 2 3; do
  for lib in $LIBS; do
    DGPPO_HIP_LIB=$(libpath $lib) timeout -k 10 100 python -u scripts/config_bench.py --only "${CFG:-LidarSpread n8}" --no-ppo 2>/dev/null \
      | python3 -c "import sys,json;[print('$lib', json.loads(l)['episode_ms']) for l in sys.stdin if l.startswith('{')]" || exit 1
  done
done
grp="GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU"
for lib in $LIBS; do
  DGPPO_HIP_LIB=$(libpath $lib) timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex rollout -d gpurun_out/abn_$lib/p1 -o run \
      --output-format csv -- python3 scripts/rollout_only.py > gpurun_out/abn_$lib.log 2>&1 || exit 1
  echo $lib; python3 scripts/pmc_summary.py gpurun_out/abn_$lib lidar_rollout_wave_kernel gpurun_out/abn_$lib.json | grep -A6 avg_per
done

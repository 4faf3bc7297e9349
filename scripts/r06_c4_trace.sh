#!/bin/bash
# kernel list of config 4's per-rank update share (512 envs, 2048-sample minibatches) and of the bench update
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c4 -o run -- \
  python3 scripts/update_time.py --env LidarBicycleTarget --envs 512 --batch 2048 --reps 1 > gpurun_out/c4.log 2>&1 || { tail gpurun_out/c4.log; exit 1; }
python3 scripts/trace_kernels.py gpurun_out/c4 32 > gpurun_out/c4_kernels.txt
python3 scripts/mb_gaps.py gpurun_out/c4 >> gpurun_out/c4_kernels.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ub -o run -- \
  python3 scripts/update_time.py --reps 1 > gpurun_out/ub.log 2>&1 || { tail gpurun_out/ub.log; exit 1; }
python3 scripts/trace_kernels.py gpurun_out/ub 32 > gpurun_out/ub_kernels.txt
cat gpurun_out/c4_kernels.txt gpurun_out/ub_kernels.txt
rm -rf gpurun_out/c4 gpurun_out/ub

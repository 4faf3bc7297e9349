#!/bin/bash
# round 6: grouped weight gradients (DGPPO_DEFER_WGRAD 1 vs 0): tests, then update time at the bench config and at
# config 4's per-rank share (512 envs, 2048-sample minibatches), interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TLIM=${TLIM:-400} TESTS="${TESTS:-tests/test_gemm_wgrad_gpu.py tests/test_update_gpu.py}" PYARGS="-x -k wgrad" bash scripts/gpu_tests.sh || exit 1
: > gpurun_out/defer_ab.jsonl
for it in 1 2; do
  for d in 1 0; do
    DGPPO_DEFER_WGRAD=$d timeout -k 10 200 python -u scripts/update_time.py --reps 5 >> gpurun_out/defer_ab.jsonl 2>/dev/null || exit 1
    DGPPO_DEFER_WGRAD=$d timeout -k 10 200 python -u scripts/update_time.py --reps 5 --env LidarBicycleTarget --envs 512 --batch 2048 >> gpurun_out/defer_ab.jsonl 2>/dev/null || exit 1
  done
done
python - <<'PY'
import json
for l in open("gpurun_out/defer_ab.jsonl"):
    d = json.loads(l); print(d["env"], d["envs"], d["knobs"], d["update_ms"], d["collect_ms"])
PY

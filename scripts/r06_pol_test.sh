#!/bin/bash
# round 6: policy-step change: rollout / nets / update parity tests, then the per-call A/B against PLIBS
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TLIM=600 TESTS="tests/test_rollout_gpu.py tests/test_nets_gpu.py tests/test_update_gpu.py tests/test_train_gpu.py" bash scripts/gpu_tests.sh | tail -4 || exit 1
PLIBS=${PLIBS:-pprev} bash scripts/r06_pol_ab.sh

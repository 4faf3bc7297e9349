#!/bin/bash
# GPU parity tests only (optionally a subset: TESTS="tests/test_nets_gpu.py -k actor").
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 ${TLIM:-900} python -u -m pytest ${TESTS:-tests} -m gpu -v --timeout 180 --timeout-method thread -p no:cacheprovider ${PYARGS:--x} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_gpu.log
exit $rc

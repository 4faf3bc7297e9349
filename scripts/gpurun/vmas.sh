cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
# VMAS parity + nets on VMAS graphs + entry points (one pytest process)
timeout -k 10 600 python -u -m pytest tests/test_vmas_gpu.py "tests/test_nets_gpu.py" -k "VMAS or vmas" -x -v --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/vmas_tests.log 2>&1
rc=$?; echo "vmas tests rc=$rc"; tail -40 gpurun_out/vmas_tests.log; exit $rc

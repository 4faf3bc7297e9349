cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
# fused policy step + register-form update forward: parity (nets / rollout tests) + timings
timeout -k 10 600 python -u -m pytest tests/test_nets_gpu.py tests/test_rollout_gpu.py -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > gpurun_out/pol_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/pol_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/policy_time.py 4096 || exit 1
DGPPO_HIP_LIB=dgppo_fov_amd/lib/libdgppo_hip_w3.so timeout -k 10 120 python -u scripts/policy_time.py 4096 || exit 1
DGPPO_POLICY_ATTN=lds timeout -k 10 120 python -u scripts/policy_time.py 4096 || exit 1
timeout -k 10 120 python -u scripts/policy_probe.py 4096 || exit 1
bash scripts/prof_mb.sh > gpurun_out/mb_run.txt 2>&1 || exit 1
grep -A3 "== Vl_fwd\|== pi_fwd\|== Vh_fwd" gpurun_out/mb_split.txt

#!/bin/bash
# round 4: first GPU run of the graph-form MFMA attention kernels: the gm-vs-row-block and oracle tests of the
# networks, then the A/B timing of one minibatch's passes and of an update
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_attn_gm_gpu.py tests/test_nets_gpu.py -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider > gpurun_out/gm1_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -30 gpurun_out/gm1_tests.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python -u scripts/attn_gm_ab.py --update > gpurun_out/gm1_ab.jsonl 2> gpurun_out/gm1_ab.err
rc2=$?; echo "ab rc=$rc2"; cat gpurun_out/gm1_ab.jsonl; tail -5 gpurun_out/gm1_ab.err
exit $rc2

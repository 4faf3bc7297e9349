#!/bin/bash
# HIP graph execution knobs on config 4's per-rank update (512 envs, 2048-sample minibatches replayed from hipGraphs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
run() { env "$@" DGPPO_PHASE_EVENTS=1 timeout -k 10 300 python3 scripts/update_time.py --env LidarBicycleTarget --envs 512 --batch 2048 --reps 5 2>/dev/null \
  | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('$*', d['collect_ms'], d['update_ms'], d['phases_ms'])"; }
run X=0 || exit 1
run DEBUG_CLR_GRAPH_PACKET_CAPTURE=1 || exit 1
run DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 || exit 1
run DEBUG_HIP_GRAPH_BATCH_SIZE=64 || exit 1
run DEBUG_HIP_FORCE_GRAPH_QUEUES=4 || exit 1
run DEBUG_HIP_FORCE_GRAPH_QUEUES=1 || exit 1

#!/bin/bash
# Interleaved A/B/C... of env-kernel library variants (scripts/build_env_variant.sh) on episode time:
#   LIBS="prev st4off" ENVS=LidarSpread:8:3:4096 bash scripts/ab_env_multi.sh   (the in-tree build always runs)
# -> gpurun_out/ab_env_multi.jsonl
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
ENVS=${ENVS:-LidarSpread:8:3:4096}
for i in 1 2 3; do
  timeout -k 10 120 python3 scripts/episode_time.py --envs $ENVS >> gpurun_out/ab_env_multi.jsonl || exit 1
  for l in $LIBS; do
    DGPPO_HIP_LIB=$PWD/dgppo_fov_amd/lib/libdgppo_hip_$l.so timeout -k 10 120 python3 scripts/episode_time.py \
      --envs $ENVS >> gpurun_out/ab_env_multi.jsonl || exit 1
  done
done
python3 - <<'PY'
import json, collections
d = collections.defaultdict(list)
for l in open("gpurun_out/ab_env_multi.jsonl"):
    r = json.loads(l); d[(r["env"], r["lib"])].append(r["episode_ms"])
for k, v in sorted(d.items()): print(k, v, "min", min(v))
PY

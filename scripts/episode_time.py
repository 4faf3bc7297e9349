"""Env-only episode time (reset + T = 128 persistent rollout, captured) for A/B runs of env-kernel builds:
prints one JSON line {lib, env, episode_ms (median of --reps), all}.  DGPPO_HIP_LIB selects the library."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgppo_fov_amd.env import make_env  # noqa: E402
from scripts.config_bench import episode_ms  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--envs", default="LidarSpread:8:3:4096")
ap.add_argument("--reps", type=int, default=15)
args = ap.parse_args()
dev = torch.device("cuda:0")
lib = os.path.basename(os.environ.get("DGPPO_HIP_LIB", "in-tree"))
for spec in args.envs.split(","):
    name, n, o, B = spec.split(":")
    env = make_env(name, int(n), num_obs=int(o), device=dev)
    t = episode_ms(env, int(B), dev, reps=args.reps)
    print(json.dumps({"lib": lib, "env": spec, "episode_ms": round(t, 4)}), flush=True)

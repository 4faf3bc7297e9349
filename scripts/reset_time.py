"""Time the states-only env reset (dgppo_env_reset_states, the bench step's first kernel) per env count:
median of 20 calls, HIP events on the launch stream.  python scripts/reset_time.py [--env LidarSpread -n 8]"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgppo_fov_amd.env import make_env  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--env", default="LidarSpread")
ap.add_argument("-n", type=int, default=8)
ap.add_argument("--obs", type=int, default=3)
args = ap.parse_args()
dev = torch.device("cuda")
env = make_env(args.env, args.n, num_obs=args.obs, device=dev)
for B in (512, 1024, 4096, 16384):
    g = env.reset_states(1, n_env=B)
    ts = []
    for i in range(25):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        env.reset_states(100 + i, n_env=B, out=g)
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts = sorted(ts[5:])
    print(json.dumps({"env": args.env, "n": args.n, "envs": B, "reset_states_us": round(ts[len(ts) // 2], 2)}), flush=True)

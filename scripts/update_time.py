"""Median DGPPO update time at the bench config (LidarSpread n8 o3, 4096 envs x 128 steps, batch 16384 -> 32
minibatches) after two warm-up updates; knobs come from the environment (DGPPO_FUSE_LN, DGPPO_FUSED_LAYER, ...).
Prints one JSON line.  --envs / --batch select other shares (e.g. --envs 512 --batch 2048: config 4's per-rank
plan), --env / -n / --obs other configs."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgppo_fov_amd.algo import make_algo  # noqa: E402
from dgppo_fov_amd.env import make_env  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--env", default="LidarSpread")
ap.add_argument("-n", type=int, default=8)
ap.add_argument("--obs", type=int, default=3)
ap.add_argument("--envs", type=int, default=4096)
ap.add_argument("--batch", type=int, default=16384)
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
dev = torch.device("cuda:0")
env = make_env(a.env, a.n, num_obs=a.obs, max_step=128, device=dev)
algo = make_algo("dgppo", env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                 action_dim=env.action_dim, n_agents=a.n, batch_size=a.batch, device=dev, train_steps=1000)
ts, cs = [], []
for it in range(2 + a.reps):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = algo.collect(algo.params, it, n_env=a.envs)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    info = algo.update(r, it)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    if it >= 2:
        cs.append((t1 - t0) * 1e3)
        ts.append((t2 - t1) * 1e3)
knobs = {k: v for k, v in os.environ.items() if k.startswith("DGPPO_")}
print(json.dumps({"env": a.env, "n": a.n, "envs": a.envs, "batch": a.batch, "update_ms": round(sorted(ts)[len(ts) // 2], 2),
                  "collect_ms": round(sorted(cs)[len(cs) // 2], 2), "update_ms_all": [round(t, 1) for t in ts],
                  "knobs": knobs, "policy_loss": round(info["policy/loss"], 6), "Vl_loss": round(info["Vl/loss"], 6),
                  "phases_ms": {k[5:]: round(v, 2) for k, v in info.items() if k.startswith("time/")}}),
      flush=True)

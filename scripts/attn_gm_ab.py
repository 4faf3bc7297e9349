"""A/B of the attention kernels on one DGPPO minibatch (LidarSpread n8, 128 envs x 128 steps = 16384 graphs):
actor eval (16-step sequences), Vl (16-step sequences) and Vh (one step) forward + backward, graph-form MFMA
kernels (dgppo_gnn_set_attn_kernel(1)) vs the row-block kernels (0), interleaved, median of 7 per pass; then one
DGPPO update at the bench config per mode (--update).  Prints one JSON line per measurement."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgppo_fov_amd import _lib  # noqa: E402
from dgppo_fov_amd.algo import make_algo  # noqa: E402
from dgppo_fov_amd.env import make_env  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--env", default="LidarSpread")
ap.add_argument("-n", type=int, default=8)
ap.add_argument("--obs", type=int, default=3)
ap.add_argument("--update", action="store_true")
a = ap.parse_args()
lib = _lib.load()
dev = torch.device("cuda:0")
T, n = 128, a.n
env = make_env(a.env, n, num_obs=a.obs, max_step=T, device=dev)
algo = make_algo("dgppo", env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                 action_dim=env.action_dim, n_agents=n, batch_size=16384, device=dev, train_steps=100)
r = algo.collect(algo.params, 0, n_env=1024)
g = algo._graphs(r.graph, torch.arange(128, device=dev)).prepare()
S, L = 128 * T // 16, 16
h = torch.randn((g.G * n, algo.Vh.carry_width), device=dev) * 0.5
acts = torch.rand((g.G * n, env.action_dim), device=dev) * 1.8 - 0.9


def run_pi():
    lp, ent, c = algo.actor.eval_seq_fwd(g, S, L, acts, algo.entropy_eps)
    algo.actor.eval_seq_bwd(c, torch.ones_like(lp) * 1e-4, torch.ones_like(ent) * 1e-4)


def run_vl():
    v, _, c = algo.Vl.seq_fwd(g, S, L)
    algo.Vl.seq_bwd(c, torch.ones_like(v) * 1e-4)


def run_vh():
    out, c = algo.Vh.fwd(g, h)
    algo.Vh.bwd(c, torch.ones_like(out) * 1e-4)


def timed(fn, reps=7):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
    return sorted(ts)[len(ts) // 2]


for m in (1, 0):  # warm both paths (workspaces, first launches)
    lib.dgppo_gnn_set_attn_kernel(m)
    for fn in (run_pi, run_vl, run_vh):
        fn()
res = {}
for rep in range(2):
    for m in (1, 0):
        lib.dgppo_gnn_set_attn_kernel(m)
        for name, fn in (("pi", run_pi), ("Vl", run_vl), ("Vh", run_vh)):
            res.setdefault((name, m), []).append(timed(fn))
for (name, m), ts in sorted(res.items()):
    print(json.dumps({"pass": name, "attn_gm": m, "ms_fwd_bwd": round(min(ts), 3), "env": a.env, "n": n}), flush=True)
if a.update:
    r4 = None
    for m in (1, 0, 1, 0):
        lib.dgppo_gnn_set_attn_kernel(m)
        r4 = algo.collect(algo.params, 3, n_env=4096)
        algo.update(r4, 0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        algo.update(r4, 1)
        torch.cuda.synchronize()
        print(json.dumps({"update_ms": round((time.perf_counter() - t0) * 1e3, 2), "attn_gm": m}), flush=True)

"""Vl (16-step sequences) and Vh (one GRU step per graph) forward + backward time of one DGPPO minibatch
(LidarSpread n8, 16384 graphs) for A/B runs of kernel knobs set through the environment (e.g. DGPPO_FUSE_LN,
the LayerNorm epilogues) or of two library builds (DGPPO_HIP_LIB)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgppo_fov_amd.algo import make_algo  # noqa: E402
from dgppo_fov_amd.env import make_env  # noqa: E402

dev = torch.device("cuda:0")
T, n = 128, 8
env = make_env("LidarSpread", n, num_obs=3, max_step=T, device=dev)
algo = make_algo("dgppo", env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                 action_dim=env.action_dim, n_agents=n, batch_size=16384, device=dev, train_steps=100)
r = algo.collect(algo.params, 0, n_env=1024)
g = algo._graphs(r.graph, torch.arange(128, device=dev))
S, L = 128 * T // 16, 16


h = torch.randn((g.G * n, 64), device=dev) * 0.5


def run_vl():
    v, _, c = algo.Vl.seq_fwd(g, S, L)
    algo.Vl.seq_bwd(c, torch.ones_like(v) * 1e-4)


def run_vh():
    out, c = algo.Vh.fwd(g, h)
    algo.Vh.bwd(c, torch.ones_like(out) * 1e-4)


res = []
for name, fn in (("Vl", run_vl), ("Vh", run_vh)):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    res.append(f"{name} fwd+bwd {(time.perf_counter() - t) / 20 * 1e3:.3f} ms")
knobs = [(k, os.path.basename(v)) for k, v in os.environ.items() if k.startswith("DGPPO_")]
print(f"knobs {knobs} " + ", ".join(res), flush=True)

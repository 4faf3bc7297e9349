"""Hash of the Vl / actor / Vh forward outputs on one LidarSpread n8 minibatch (A/B bit-identity of kernel knobs:
run twice with different DGPPO_* settings and compare the printed digests).  GPU only."""
import hashlib
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgppo_fov_amd.algo import make_algo  # noqa: E402
from dgppo_fov_amd.env import make_env  # noqa: E402

dev = torch.device("cuda:0")
T, n = 128, 8
env = make_env("LidarSpread", n, num_obs=3, max_step=T, device=dev)
algo = make_algo("dgppo", env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                 action_dim=env.action_dim, n_agents=n, batch_size=16384, device=dev, train_steps=100)
r = algo.collect(algo.params, 0, n_env=256)
g = algo._graphs(r.graph, torch.arange(128, device=dev))
S, L = 128 * T // 16, 16
v, _, _ = algo.Vl.seq_fwd(g, S, L)
h = torch.randn((g.G * n, 64), device=dev, generator=torch.Generator(device=dev).manual_seed(0)) * 0.5
vh, _ = algo.Vh.fwd(g, h)
torch.cuda.synchronize()
d = hashlib.sha256()
for t in (v, vh, r.actions, r.log_pis):
    d.update(t.detach().float().cpu().numpy().tobytes())
print("digest", d.hexdigest()[:16], {k: v for k, v in os.environ.items() if k.startswith("DGPPO_")}, flush=True)

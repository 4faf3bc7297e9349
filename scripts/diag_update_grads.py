"""Diagnostic: per-tensor gradient error of one DGPPO minibatch, GPU vs float64 oracle, next to the
error of the same oracle evaluated in float32 (the natural fp32 noise floor)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_update_gpu import _host, _net_trees, _walk  # noqa: E402
from dgppo_fov_amd.algo import make_algo  # noqa: E402
from dgppo_fov_amd.env import make_env  # noqa: E402
from oracle import nets_t as R  # noqa: E402

eid, n, obs = os.environ.get("ENV_ID", "LidarSpread"), 3, 2
B, T, L = 4, 32, 16
cuda = torch.device("cuda:0")
env = make_env(eid, n, num_obs=obs, max_step=T, device=cuda)
algo = make_algo("dgppo", env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                 action_dim=env.action_dim, n_agents=n, batch_size=B * T, rnn_step=L, train_steps=100, seed=1,
                 device=cuda)
roll = algo.collect(algo.params, 7, n_env=B)
pa, pl, ph = _net_trees(algo)
algo.trace = {}
algo.update(roll, 60)
tr = algo.trace
hr, hd = _host(roll, n), _host(tr["det"], n)
(mb,) = tr["mb"]
algo.grad_flat.copy_(mb["grad"])
gpu = _net_trees(algo, grad=True)
res = {}
for dt in (torch.float64, torch.float32):
    R.T64 = dt
    ts = [R.to_t(x, requires_grad=True) for x in (pa, pl, ph)]
    R.dgppo_minibatch_grads(*ts, hr, hd, np.asarray(mb["envs"]), tr["Ql"].double().cpu().numpy(),
                            tr["Qh_det"].double().cpu().numpy(), tr["A"].double().cpu().numpy(), n, L,
                            algo.entropy_eps.cpu().numpy(), algo.clip_eps, algo.coef_ent)
    res[dt] = [R.grads(t) for t in ts]
for tag, g, r64, r32 in zip(("actor", "Vl", "Vh"), gpu, res[torch.float64], res[torch.float32]):
    for (path, a, b), (_, c, _) in zip(_walk(g, r64), _walk(r32, r64)):
        b = np.asarray(b, np.float64)
        e_gpu = np.abs(np.asarray(a, np.float64) - b).max()
        e_32 = np.abs(np.asarray(c, np.float64) - b).max()
        print(f"{tag:5s} {path:40s} scale {np.abs(b).max():.3e}  gpu {e_gpu:.3e}  ref32 {e_32:.3e}  ratio {e_gpu/max(e_32,1e-30):.2f}")

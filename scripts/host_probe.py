"""Host-side launch time of the update's minibatch step (Python + launch API, no synchronisation) against the
update's wall time at the bench config: if the host needs as long as the GPU, the minibatches are host-bound."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgppo_fov_amd.algo import make_algo  # noqa: E402
from dgppo_fov_amd.env import make_env  # noqa: E402

dev = torch.device("cuda:0")
env = make_env("LidarSpread", 8, num_obs=3, max_step=128, device=dev)
algo = make_algo("dgppo", env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                 action_dim=env.action_dim, n_agents=8, batch_size=16384, device=dev, train_steps=1000)
acc = {"t": 0.0, "n": 0}
orig = algo._mb_body


def timed(*a, **k):
    t = time.perf_counter()
    out = orig(*a, **k)
    acc["t"] += time.perf_counter() - t
    acc["n"] += 1
    return out


algo._mb_body = timed
for it in range(4):
    r = algo.collect(algo.params, it, n_env=4096)
    torch.cuda.synchronize()
    acc["t"], acc["n"] = 0.0, 0
    t0 = time.perf_counter()
    algo.update(r, it)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    print(f"update {wall * 1e3:.1f} ms wall; host time in {acc['n']} minibatch bodies {acc['t'] * 1e3:.1f} ms "
          f"({acc['t'] / max(acc['n'], 1) * 1e3:.2f} ms each)", flush=True)

"""LidarOmniTarget DGPPO collect at the BASELINE-style config (n=8, 3 obstacles, 4096 envs, T=128): wall time
of one collect with the fused policy step (DGPPO_FUSED_POLICY=1, default) or the unfused layer chain (=0)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgppo_fov_amd.algo import make_algo  # noqa: E402
from dgppo_fov_amd.env import make_env  # noqa: E402

dev = torch.device("cuda:0")
B = int(os.environ.get("N_ENV", "4096"))
env = make_env("LidarOmniTarget", 8, num_obs=3, device=dev)
algo = make_algo("dgppo", env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                 action_dim=env.action_dim, n_agents=8, batch_size=16384, device=dev, train_steps=100)
for it in range(4):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    r = algo.collect(algo.params, it, n_env=B)
    torch.cuda.synchronize()
    print(f"fused={os.environ.get('DGPPO_FUSED_POLICY', '1')} collect {1e3 * (time.perf_counter() - t0):.1f} ms "
          f"reward {r.rewards.sum(1).mean().item():.4f}", flush=True)

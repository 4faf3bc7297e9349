"""Run collect + update of DGPPO on a small config and print the info dict + timings."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgppo_fov_amd.algo import make_algo  # noqa: E402
from dgppo_fov_amd.env import make_env  # noqa: E402

env_id = os.environ.get("ENV_ID", "LidarSpread")
n = int(os.environ.get("N_AGENTS", "3"))
obs = int(os.environ.get("N_OBS", "2"))
B = int(os.environ.get("N_ENV", "16"))
T = int(os.environ.get("T", "32"))
bs = int(os.environ.get("BATCH", str(B * T // 2)))
iters = int(os.environ.get("ITERS", "2"))
MARK = os.environ.get("MARK_UPDATE", "1") == "1"
dev = torch.device("cuda:0")
env = make_env(env_id, n, num_obs=obs, max_step=T, device=dev)
algo = make_algo("dgppo", env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                 action_dim=env.action_dim, n_agents=n, batch_size=bs, device=dev, train_steps=100)
for it in range(iters):
    t0 = time.perf_counter()
    r = algo.collect(algo.params, it, n_env=B)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if MARK:
        torch.cuda._sleep(1000)  # a `spin_kernel` dispatch marks where the update starts (scripts/mfma_util.py)
    info = algo.update(r, it)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"iter {it}: collect {1e3*(t1-t0):.1f} ms, update {1e3*(t2-t1):.1f} ms, reward {r.rewards.sum(1).mean().item():.4f}")
    print({k: round(v, 5) for k, v in info.items()})

import os, sys, time
import torch
sys.path.insert(0, "/root/repo")
from dgppo_fov_amd.algo import make_algo
from dgppo_fov_amd.env import make_env
dev = torch.device("cuda:0")
env = make_env("LidarOmniTarget", 8, num_obs=3, max_step=128, device=dev)
algo = make_algo("dgppo", env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                 action_dim=env.action_dim, n_agents=8, batch_size=16384, device=dev, train_steps=100)
for it in range(3):
    torch.cuda.synchronize(); t0 = time.perf_counter()
    r = algo.collect(algo.params, it, n_env=4096)
    torch.cuda.synchronize(); print("collect ms", (time.perf_counter() - t0) * 1e3, flush=True)

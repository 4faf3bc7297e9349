"""Minimal driver for rocprofv3 PMC passes: reset + N eager env steps of the bench workload."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgppo_fov_amd.env import make_env  # noqa: E402

env_id = os.environ.get("ENV_ID", "LidarSpread")
n = int(os.environ.get("N_AGENTS", "8"))
obs = int(os.environ.get("N_OBS", "3"))
B = int(os.environ.get("N_ENV", "4096"))
steps = int(os.environ.get("N_STEPS", "20"))
dev = torch.device("cuda:0")
env = make_env(env_id, n, num_obs=obs, device=dev)
g = env.reset(key=1, n_env=B)
a = torch.rand(B, n, 2, device=dev) * 2 - 1
for _ in range(steps):
    g = env.step(g, a).graph
torch.cuda.synchronize()
print("done", env_id, n, obs, B, steps)

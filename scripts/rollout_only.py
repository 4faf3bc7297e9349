"""Minimal driver for rocprofv3 passes on the persistent env rollout: the bench workload's env-only
rollout (states-only reset + one dgppo_env_rollout launch of T=128 steps), eager, N_REPS times."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgppo_fov_amd.env import make_env  # noqa: E402
from dgppo_fov_amd.trainer.rollout import RolloutEngine  # noqa: E402

env_id = os.environ.get("ENV_ID", "LidarSpread")
n = int(os.environ.get("N_AGENTS", "8"))
obs = int(os.environ.get("N_OBS", "3"))
B = int(os.environ.get("N_ENV", "4096"))
reps = int(os.environ.get("N_REPS", "6"))
dev = torch.device("cuda:0")
env = make_env(env_id, n, num_obs=obs, device=dev)
eng = RolloutEngine(env, B, 128, dev)
eng.actions.uniform_(-1, 1)
for r in range(reps):
    eng.run(key=r)
torch.cuda.synchronize()
print("done", env_id, n, obs, B, reps)

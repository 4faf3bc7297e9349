"""A/B timing of the env-step kernels (wave-per-env vs workgroup-per-env) at the bench workload:
average launch time from HIP events around back-to-back launches on the launch stream."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgppo_fov_amd import _lib  # noqa: E402
from dgppo_fov_amd.env import make_env  # noqa: E402

dev = torch.device("cuda:0")
lib = _lib.load()
for eid, n, obs, B in [("LidarSpread", 8, 3, 4096), ("LidarBicycleTarget", 8, 3, 4096), ("LidarTarget", 8, 3, 4096)]:
    env = make_env(eid, n, num_obs=obs, device=dev)
    g = env.reset(key=1, n_env=B)
    a = torch.rand(B, n, 2, device=dev) * 2 - 1
    for mode, name in ((1, "block"), (0, "wave")):
        lib.dgppo_env_set_step_kernel(mode)
        gg = g
        for _ in range(20):
            gg = env.step(gg, a).graph
        s = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(s)
        for _ in range(200):
            gg = env.step(gg, a).graph
        e1.record(s)
        torch.cuda.synchronize()
        print(f"{eid:20s} {name:6s} {e0.elapsed_time(e1) / 200 * 1e3:8.2f} us/step (incl. python launch)", flush=True)
lib.dgppo_env_set_step_kernel(0)

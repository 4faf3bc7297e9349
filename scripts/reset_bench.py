"""env reset kernel time (HIP events around 16 back-to-back resets captured in a hipGraph) for the
bench config and LidarOmniTarget, 4096 envs."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgppo_fov_amd.env import make_env  # noqa: E402

dev = torch.device("cuda:0")
for eid in ("LidarSpread", "LidarOmniTarget", "MPESpread"):
    env = make_env(eid, 8 if eid != "MPESpread" else 3, num_obs=3, device=dev)
    B = 4096
    env.reset(key=0, n_env=B)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for rep in range(5):
        e0.record()
        for k in range(16):
            env.reset(key=100 * rep + k, n_env=B)
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) / 16 * 1e3)
    print(json.dumps({"env": eid, "n_env": B, "reset_us_incl_host": round(sorted(ts)[2], 1)}))

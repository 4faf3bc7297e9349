import json, sys, torch
sys.path.insert(0, "/root/repo")
from dgppo_fov_amd.env import make_env
dev = torch.device("cuda:0")
for (eid, n, o) in [("LidarSpread", 8, 3), ("LidarSpread", 8, 0), ("LidarSpread", 1, 3), ("LidarSpread", 4, 3)]:
    env = make_env(eid, n, num_obs=o, device=dev)
    B = 4096
    env.reset(key=0, n_env=B); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for rep in range(5):
        e0.record()
        for k in range(16): env.reset(key=100 * rep + k, n_env=B)
        e1.record(); e1.synchronize(); ts.append(e0.elapsed_time(e1) / 16 * 1e3)
    print(json.dumps({"env": eid, "n": n, "obs": o, "reset_us": round(sorted(ts)[2], 1)}))

"""LidarOmniTarget env-step kernel timing (n=8, 3 obstacles, 4096 envs): average launch time from
HIP events around 64 back-to-back launches captured in a hipGraph, and the algorithmic-bytes
roofline (reads: agent + goal rows (7 floats), all 64 current hits (2), 3 obstacle records (16),
actions (3); writes: nodes (81 x 10), states (81 x 7), edges (136 x 10), receivers / senders
(136 each), reward, cost (8 x 5))."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgppo_fov_amd import _lib  # noqa: E402
from dgppo_fov_amd.env import make_env  # noqa: E402

n, O, B = 8, 3, 4096
N, E, k = 2 * n + n * 8 + 1, n * n + n + n * 8, 8
BYTES = 4 * ((2 * n * 7 + n * k * 2 + O * 16 + n * 3) + (N * 10 + N * 7 + E * 10 + 2 * E + 1 + n * 5))
dev = torch.device("cuda:0")
env = make_env("LidarOmniTarget", n, num_obs=O, device=dev)
g = env.reset(key=1, n_env=B)
a = torch.rand(B, n, 3, device=dev) * 2 - 1
ob = g.env_states.obstacle.packed
outs = [env.empty_graph((B,), dev) for _ in range(2)]
outs = [env._assemble(o.nodes, o.edges, o.states, o.receivers, o.senders, ob) for o in outs]
rew = torch.empty(B, device=dev)
cost = torch.empty(B, n, 5, device=dev)


def loop(m=64):
    cur = g
    for i in range(m):
        cur = env.step_into(cur if i == 0 else outs[(i - 1) & 1], a, outs[i & 1], rew, cost)


def measure():
    loop()
    torch.cuda.synchronize()
    cg = torch.cuda.CUDAGraph()
    with torch.cuda.graph(cg):
        loop()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(7):
        e0.record()
        cg.replay()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) / 64 * 1e3)
    return sorted(ts)[len(ts) // 2]


lib = _lib.load()
for mode, name in ((0, "wv::lidar_step_wave_kernel<OMNI,TARGET,7,3>"), (1, "omni_step_kernel<256>")):
    lib.dgppo_env_set_step_kernel(mode)
    us = measure()
    gbs = BYTES * B / us / 1e3
    print(json.dumps({"env": "LidarOmniTarget", "n": n, "n_obs": O, "n_env": B, "kernel": name,
                      "us_per_launch": round(us, 2), "env_steps_per_s": round(B / us * 1e6, 1),
                      "bytes_per_env_step": BYTES, "achieved_GBs": round(gbs, 1), "frac_of_8TBs": round(gbs / 8000, 4)}))
lib.dgppo_env_set_step_kernel(0)

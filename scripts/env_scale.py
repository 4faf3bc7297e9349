"""Env-step kernel time vs batch size (is the wave kernel throughput- or latency-bound?):
average launch time from HIP events around back-to-back launches captured in a hipGraph."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgppo_fov_amd import _lib  # noqa: E402
from dgppo_fov_amd.env import make_env  # noqa: E402

dev = torch.device("cuda:0")
env = make_env("LidarSpread", 8, num_obs=3, device=dev)
lib = _lib.load()
for mode, B in [(m, b) for m in (0, 1) for b in (512, 1024, 2048, 4096, 8192, 16384)]:
    lib.dgppo_env_set_step_kernel(mode)  # 0: wave per env, 1: workgroup per env
    g = env.reset(key=1, n_env=B)
    a = torch.rand(B, 8, 2, device=dev) * 2 - 1
    ob = g.env_states.obstacle.packed
    outs = [env.empty_graph((B,), dev) for _ in range(2)]
    outs = [env._assemble(o.nodes, o.edges, o.states, o.receivers, o.senders, ob) for o in outs]
    rew = torch.empty(B, device=dev)
    cost = torch.empty(B, 8, 2, device=dev)

    def loop(n=64):
        cur = g
        for i in range(n):
            cur = env.step_into(cur if i == 0 else outs[(i - 1) & 1], a, outs[i & 1], rew, cost)

    loop()
    torch.cuda.synchronize()
    cg = torch.cuda.CUDAGraph()
    with torch.cuda.graph(cg):
        loop()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(5):
        e0.record()
        cg.replay()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) / 64 * 1e3)
    ts.sort()
    us = ts[len(ts) // 2]
    print(f"mode={mode} B={B:6d}  {us:8.2f} us/step  {B / us:8.1f} env-steps/us  {8856 * B / us / 1e3:7.1f} GB/s", flush=True)

"""Phase timestamps of the fused policy step (diagnostic library, `make probe`: every workgroup's thread 0
writes s_memrealtime (100 MHz) at each PROBE(k) into h_out viewed as uint64[grid][32]).  Prints the mean
per-workgroup time of each phase and the spread of workgroup start times, for LidarSpread n=8 obs=3 at
4096 envs.  Run with DGPPO_HIP_LIB=dgppo_fov_amd/lib/libdgppo_hip_probe.so (set below when unset)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("DGPPO_HIP_LIB", os.path.join(ROOT, "dgppo_fov_amd", "lib", "libdgppo_hip_probe.so"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from dgppo_fov_amd.algo import make_algo  # noqa: E402
from dgppo_fov_amd.env import make_env  # noqa: E402
from dgppo_fov_amd.nn.layers import GraphBatch  # noqa: E402

PH = [(0, 1, "loads: cand / raw rows / carries / params, pair tables, pair gathers"),
      (1, 2, "layer 0 [QT|beta] GEMM + operands"), (2, 3, "layer 0 attention (2 sub-rounds)"),
      (3, 4, "layer 0 message + update GEMMs"), (4, 5, "layer 1 weight loads + [QT|beta] GEMM"),
      (5, 6, "layer 1 attention (pre-transform MFMA)"), (6, 7, "layer 1 message + update GEMMs"),
      (7, 12, "head / GRU / ScaleHid weight fragment loads"), (12, 8, "MLP head (2 Dense + LN + ReLU)"),
      (8, 9, "GRU"), (9, 10, "ScaleHid"), (10, 11, "mean / std / TanhNormal")]


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    dev = torch.device("cuda:0")
    env = make_env("LidarSpread", 8, num_obs=3, device=dev)
    algo = make_algo("dgppo", env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                     action_dim=env.action_dim, n_agents=8, batch_size=16384, device=dev)
    g = env.reset(1, n_env=B)
    gb = GraphBatch.from_graph(g, env)
    n = 8
    grid = B * n // 16
    h = torch.zeros((B * n, 64), device=dev)
    hout = torch.zeros((max(B * n, grid * 16), 64), device=dev)
    noise = torch.randn((B * n, 2), device=dev)
    out = []
    for rep in range(6):
        algo.actor.act(gb, h, 1, noise=noise, h_out=hout, prepare=rep == 0)
        torch.cuda.synchronize()
        if rep:
            ts = hout.view(torch.int64).view(-1)[: grid * 32].view(grid, 32).cpu().numpy().astype(np.float64)
            out.append(ts)
    ts = np.stack(out)  # (reps, grid, 32) ticks of 10 ns
    res = {"B": B, "workgroups": grid, "phases_us": {}}
    for a, b, name in PH:
        res["phases_us"][name] = round(float(np.mean(ts[:, :, b] - ts[:, :, a])) * 0.01, 2)
    res["workgroup_total_us"] = round(float(np.mean(ts[:, :, 11] - ts[:, :, 0])) * 0.01, 2)
    res["kernel_span_us"] = round(float(np.mean(ts[:, :, 11].max(1) - ts[:, :, 0].min(1))) * 0.01, 2)
    res["start_spread_us"] = round(float(np.mean(ts[:, :, 0].max(1) - ts[:, :, 0].min(1))) * 0.01, 2)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()

"""Per-call time of the fused policy step (ActorNet.act, mode 1) for LidarSpread n=8 obs=3 at B envs:
HIP events around 50 back-to-back calls on the current stream.  DGPPO_HIP_LIB selects another build (e.g. lib/libdgppo_hip_w3.so)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from dgppo_fov_amd.algo import make_algo  # noqa: E402
from dgppo_fov_amd.env import make_env  # noqa: E402
from dgppo_fov_amd.nn.layers import GraphBatch  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    eid = os.environ.get("ENV_ID", "LidarSpread")
    n, obs = int(os.environ.get("N_AGENTS", 8)), int(os.environ.get("N_OBS", 3))
    dev = torch.device("cuda:0")
    env = make_env(eid, n, num_obs=obs, device=dev)
    algo = make_algo("dgppo", env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                     action_dim=env.action_dim, n_agents=n, batch_size=16384, device=dev)
    g = env.reset(1, n_env=B)
    gb = GraphBatch.from_graph(g, env).prepare()
    h = torch.randn((B * n, 64), device=dev) * 0.3
    hout = torch.empty((B * n, 64), device=dev)
    noise = torch.randn((B * n, env.action_dim), device=dev)
    for rep in range(3):
        a, lp, _ = algo.actor.act(gb, h, 1, noise=noise, h_out=hout, prepare=rep == 0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(5):
        e0.record()
        for _ in range(50):
            algo.actor.act(gb, h, 1, noise=noise, h_out=hout, prepare=False)
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) / 50 * 1e3)
    a, lp, h2 = algo.actor.act(gb, h, 1, noise=noise, h_out=hout, prepare=False)
    torch.cuda.synchronize()
    print(json.dumps({"env": eid, "n": n, "B": B, "attn": "reg",
                      "lib": os.path.basename(os.environ.get("DGPPO_HIP_LIB", "libdgppo_hip.so")),
                      "act_us_median": round(sorted(ts)[2], 2), "act_us_all": [round(t, 2) for t in ts],
                      "checksum": [float(a.double().sum()), float(lp.double().sum()), float(h2.double().sum())]}))


if __name__ == "__main__":
    main()

"""Per-GPU throughput of every BASELINE.json config on one MI355X (the bench line covers configs[2]).

For each config: the env-step kernel (average launch time from HIP events around 64 back-to-back
launches captured in a hipGraph, ping-ponging two graph buffers), one env-only episode (reset + T = 128
steps through RolloutEngine, captured: the persistent rollout kernel where the library has it for the
config, else the step kernel looped inside the call) and, unless --no-ppo, one DGPPO
collect + update at batch 16384 / rnn_step 16 (second call timed; the first captures graphs and grows
workspaces).  Multi-GPU configs are measured at their per-GPU share (env-sharded, weak scaling).
Random-init networks, synthetic resets and uniform random actions."""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgppo_fov_amd.algo import make_algo  # noqa: E402
from dgppo_fov_amd.env import make_env  # noqa: E402
from dgppo_fov_amd.trainer.rollout import RolloutEngine  # noqa: E402

# (label, env, n, obs, envs per GPU)
CONFIGS = [
    ("MPESpread n3 o3 x1024", "MPESpread", 3, 3, 1024),
    ("LidarSpread n8 o3 x4096", "LidarSpread", 8, 3, 4096),
    ("LidarBicycleTarget n8 o3 x4096/GPU (8-GPU config)", "LidarBicycleTarget", 8, 3, 4096),
    # config 4's strong-scaling share: 4096 envs over 8 GPUs = 512 per GPU; the global 16384-sample minibatch is
    # 2048 samples per rank (batch 2048 here gives the per-rank plan: 32 minibatches of 16 envs; no all-reduce)
    ("LidarBicycleTarget n8 o3 x512/GPU (config 4 strong share, 2048-sample rank minibatch)", "LidarBicycleTarget", 8,
     3, 512, 2048),
    # config 5's share: 8192 envs over 8 GPUs = 1024 per GPU; minibatch_plan at world 8 gives each rank 64 minibatches
    # of 2048 samples (batch 2048 here reproduces that per-rank plan on one GPU; no all-reduce)
    ("LidarSpread n32 o8 x1024/GPU (config 5 share, 64 x 2048-sample rank minibatches)", "LidarSpread", 32, 8, 1024,
     2048),
    ("LidarOmniTarget n8 o3 x4096", "LidarOmniTarget", 8, 3, 4096),
    # env variants (no BASELINE config names them): same per-GPU shapes as their base envs
    ("LidarLine n6 o3 x4096 (variant; n = 8 does not fit the landmarks in the default area)", "LidarLine", 6, 3, 4096),
    ("MPELine n3 o3 x1024 (variant)", "MPELine", 3, 3, 1024),
    ("MPEFormation n3 o3 x1024 (variant)", "MPEFormation", 3, 3, 1024),
    ("MPECorridor n3 x1024 (variant, 2 fixed obstacles)", "MPECorridor", 3, 2, 1024),
    ("MPEConnectSpread n3 x1024 (variant, 1 fixed obstacle)", "MPEConnectSpread", 3, 1, 1024),
    # VMAS contact physics (no BASELINE config names them): the MPE-sized batch and a 4x larger one
    ("VMASWheel n3 x1024", "VMASWheel", 3, 0, 1024),
    ("VMASWheel n3 x4096", "VMASWheel", 3, 0, 4096),
    ("VMASReverseTransport n3 x1024", "VMASReverseTransport", 3, 0, 1024),
    ("VMASReverseTransport n3 x4096", "VMASReverseTransport", 3, 0, 4096),
]


def step_us(env, B, dev, m=64):
    g = env.reset(key=1, n_env=B)
    a = torch.rand(B, env.num_agents, env.action_dim, device=dev) * 2 - 1
    ob = env._obstacles_of(g)  # Lidar: rectangle records; VMAS: per-env records; MPE: None (in the states)
    outs = [env.empty_graph((B,), dev) for _ in range(2)]
    outs = [env._assemble(o.nodes, o.edges, o.states, o.receivers, o.senders, ob) for o in outs]
    rew = torch.empty(B, device=dev)
    cost = torch.empty(B, env.num_agents, env.n_cost, device=dev)

    def loop():
        for i in range(m):
            env.step_into(g if i == 0 else outs[(i - 1) & 1], a, outs[i & 1], rew, cost)

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
        ts.append(e0.elapsed_time(e1) / m * 1e3)
    return sorted(ts)[len(ts) // 2]


def episode_ms(env, B, dev, T=128, reps=10):
    eng = RolloutEngine(env, B, T, dev, lanes=1)
    eng.actions.uniform_(-1.0, 1.0)
    eng.capture()
    for w in range(3):
        eng.run(key=w)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for k in range(reps):
        e0.record()
        eng.run(key=100 + k)
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    return sorted(ts)[len(ts) // 2]


def ppo_ms(env, B, dev, batch=16384, reps=1):
    """Median over `reps` timed collect + update iterations (after one untimed one)."""
    algo = make_algo("dgppo", env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                     action_dim=env.action_dim, n_agents=env.num_agents, batch_size=batch, rnn_step=16, seed=0,
                     device=dev, train_steps=1000)
    r = algo.collect(algo.params, 0, n_env=B)
    algo.update(r, 0)
    torch.cuda.synchronize()
    cs, us = [], []
    for k in range(reps):
        t0 = time.perf_counter()
        r = algo.collect(algo.params, 1 + k, n_env=B)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        algo.update(r, 1 + k)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        cs.append((t1 - t0) * 1e3)
        us.append((t2 - t1) * 1e3)
    return sorted(cs)[len(cs) // 2], sorted(us)[len(us) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--no-ppo", action="store_true")
    ap.add_argument("--only", default="", help="run only the configs whose label contains this string")
    ap.add_argument("--step-kernel", default="auto", choices=["auto", "block"],
                    help="block: force the workgroup-per-env env kernels (dgppo_env_set_step_kernel(1))")
    ap.add_argument("--reps", type=int, default=1, help="timed collect + update iterations (median)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    if args.step_kernel == "block":
        from dgppo_fov_amd import _lib
        _lib.load().dgppo_env_set_step_kernel(1)
    for label, eid, n, obs, B, *rest in CONFIGS:
        batch = rest[0] if rest else 16384
        if args.only not in label:
            continue
        env = make_env(eid, n, num_obs=obs, max_step=128, device=dev)
        us = step_us(env, B, dev)
        row = {"config": label, "env": eid, "n": n, "n_obs": obs, "envs_per_gpu": B, "env_step_us": round(us, 2),
               "env_steps_per_s": round(B / us * 1e6, 1), "step_kernel": args.step_kernel,
               "update_graph": os.environ.get("DGPPO_UPDATE_GRAPH", "0")}
        ep = episode_ms(env, B, dev)
        row.update({"episode_ms": round(ep, 3), "episode_env_steps_per_s": round(B * 128 / ep * 1e3, 1)})
        if not args.no_ppo:
            c, u = ppo_ms(env, B, dev, batch, args.reps)
            row.update({"collect_ms": round(c, 2), "update_ms": round(u, 2), "batch_size": batch,
                        "minibatches": B * 128 // batch})
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()

"""Benchmark of the DGPPO hot path on MI355X (driver contract: one JSON line from rank 0).

Workload (BASELINE.json metric "env-steps/sec + PPO-updates/sec, LidarSpread n=8 x4096 envs"):
LidarSpread, n=8 agents, 3 obstacles, 32 rays, 4096 parallel envs per GPU.  One bench "step" is
one episode of the rollout hot path: env reset + T=128 fused env steps over all 4096 envs (stepped as
2 slices of 2048 envs on 2 HIP streams inside one hipGraph, DGPPO_BENCH_LANES), with
synthetic random actions already resident in HBM, writing the full (B, T+1) graph rollout buffer
(the reference's `collect` minus the policy).  `value` = env transitions per second over all
ranks.  The "ppo" object times full DGPPO training iterations at the same config (policy rollout
+ update, batch 16384, rnn_step 16): `ppo_updates_per_s` = update() calls per second.  Multi-GPU: envs are sharded (rank r owns envs [r*B, (r+1)*B)), no data-path collective —
weak scaling.

roofline: the dominant kernel is the env-step kernel (HBM-bound).  Algorithmic bytes per env
transition = 8,856 B; per launch = 8,856 * 4096.  Its average duration is measured
live with HIP events around back-to-back step launches on the launch stream.
cpu_baseline: the NumPy oracle (oracle/env.py, single thread) on a bounded sample.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "env-steps/sec + PPO-updates/sec, LidarSpread n=8 ×4096 envs, 1/2/4/8 GPU"
ENV_ID, N_AGENTS, N_OBS, B_PER_GPU, T = "LidarSpread", 8, 3, 4096, 128
BYTES_PER_ENV_STEP = 8856  # SURVEY.md §8(d), LidarSpread n8 O3
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


def cpu_baseline(budget_s=12.0):
    """NumPy oracle (1 thread, vectorised over envs) on a bounded sample of the same workload."""
    from oracle import env as O

    spec = O.Spec(ENV_ID, N_AGENTS, N_OBS)
    Bs = 1024
    ag, gl, third = O.env_reset(spec, 1, Bs)
    g = O.initial_graph(spec, ag, gl, third)
    rng = np.random.default_rng(0)
    states = g["states"]
    n_steps = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < budget_s and n_steps < T:
        a = rng.uniform(-1, 1, (Bs, N_AGENTS, 2)).astype(np.float32)
        out = O.env_step(spec, states, third, a)
        states = out["states"]
        n_steps += 1
    dt = time.perf_counter() - t0
    return {"value": round(Bs * n_steps / dt, 1), "unit": "env-steps/s", "cores": 1, "kind": "port",
            "sample": f"oracle/env.py NumPy fp32, {Bs} envs x {n_steps} LidarSpread n=8 steps "
                      f"({dt:.1f} s, reset excluded), 1 thread"}


def read_pmc_traffic():
    fn = os.path.join(ROOT, "profiles", "env_step_pmc.json")
    if os.path.exists(fn):
        try:
            return json.load(open(fn)).get("hbm_bytes_per_launch")
        except Exception:
            return None
    return None


def read_mfma_pmc():
    """Executed-MFMA utilisation from the committed PMC profile (scripts/mfma_pmc.sh): SQ_INSTS_VALU_MFMA_MOPS_F32
    x 512 per kernel family over one collect + update, against the fp32 MFMA peak."""
    fn = os.path.join(ROOT, "profiles", "r01_mfma_util.json")
    if not os.path.exists(fn):
        return None
    try:
        d = json.load(open(fn))
        fam = d["families"]
        gemm_t = sum(fam[k]["time_ms"] for k in ("gemm_rows", "gemm_wgrad") if k in fam)
        gemm_f = sum(fam[k]["mfma_tflop"] for k in ("gemm_rows", "gemm_wgrad") if k in fam)
        return {"source": "profiles/r01_mfma_util.json (rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F32)",
                "gnn_gemm_executed_tflops": round(gemm_f / gemm_t * 1e3, 2),
                "gnn_gemm_frac_of_peak": round(gemm_f / gemm_t * 1e3 / FP32_MFMA_PEAK_TFLOPS, 4),
                "window_executed_tflops": d["total_mfma_tflops_over_window"],
                "window_frac_of_peak": round(d["total_mfma_tflops_over_window"] / FP32_MFMA_PEAK_TFLOPS, 4)}
    except Exception:
        return None


PPO_BATCH, RNN_STEP = 16384, 16  # BASELINE.md synthetic-input plan (batch_size, rnn_step)
# SURVEY.md §8(d) official algorithmic flops (minimal node-level projection formulation), LidarSpread n8
# B4096: one PPO update (det rollout excluded: prepass + SGD, fwd+bwd = 3x fwd) and the two rollouts'
# actor inference; MFMA% = flops / (t * 157.3 TF * n_gpu)
UPDATE_TFLOP_PER_4096_ENVS, ROLLOUT_TFLOP_PER_4096_ENVS = 22.1, 5.3
FP32_MFMA_PEAK_TFLOPS = 157.3


def ppo_bench(env, dev, world, rank, iters):
    """DGPPO training iterations at the bench config: collect (policy rollout, 4096 envs x T=128 in
    one hipGraph) + update (det rollout, Vl/Vh prepass, GAE, advantages, 32 minibatches x
    [Vl, Vh, policy fwd+bwd, one grad all-reduce, clip + Adam]).  Random-init nets, synthetic envs.
    Max over ranks of the wall time between barriers."""
    from dgppo_fov_amd.algo import make_algo
    from dgppo_fov_amd.nn import kernels as K

    algo = make_algo("dgppo", env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                     action_dim=env.action_dim, n_agents=N_AGENTS, batch_size=PPO_BATCH * world, rnn_step=RNN_STEP,
                     seed=0, device=dev, train_steps=1000)
    r = algo.collect(algo.params, 0, n_env=B_PER_GPU)
    algo.update(r, 0)  # warm-up: captures the deterministic-rollout graph, grows workspaces
    K.GEMM_LOG = []
    algo.update(r, 0)
    gemm_flops = sum(2.0 * M * N * Kd * b for (M, N, Kd, b, *_rest) in K.GEMM_LOG)
    K.GEMM_LOG = None
    t_col = t_upd = 0.0
    for it in range(iters):
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        r = algo.collect(algo.params, 100 + it, n_env=B_PER_GPU)
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        algo.update(r, it)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        t2 = time.perf_counter()
        t_col += t1 - t0
        t_upd += t2 - t1
    t = torch.tensor([t_col, t_upd], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    t_col, t_upd = (float(x) / iters for x in t.tolist())
    upd_tf = UPDATE_TFLOP_PER_4096_ENVS * (B_PER_GPU / 4096) * world + ROLLOUT_TFLOP_PER_4096_ENVS / 2 * (
        B_PER_GPU / 4096) * world  # the update runs the deterministic rollout too
    return {"updates_per_s": round(1.0 / t_upd, 4), "update_ms": round(t_upd * 1e3, 2),
            "update_roofline": {"bound": "mfma", "algorithmic_tflop": round(upd_tf, 2),
                                "achieved": round(upd_tf / t_upd, 2), "peak": FP32_MFMA_PEAK_TFLOPS * world,
                                "unit": "TFLOP/s", "frac": round(upd_tf / t_upd / (FP32_MFMA_PEAK_TFLOPS * world), 4),
                                "flops_source": "SURVEY.md 8(d): 22.1 TF per update + 2.65 TF det-rollout inference"},
            "collect_ms": round(t_col * 1e3, 2),
            "collect_env_steps_per_s": round(B_PER_GPU * T * world / t_col, 1),
            "iters": iters, "batch_size": PPO_BATCH * world, "rnn_step": RNN_STEP, "epoch_ppo": 1,
            "minibatches": B_PER_GPU * T * world // (PPO_BATCH * world),
            "gemm_tflop_per_update": round(gemm_flops / 1e12, 3),
            "gemm_tflops_over_update": round(gemm_flops / t_upd / 1e12, 3), "fp32_mfma_peak_tflops": 157.3,
            "mfma_pmc": read_mfma_pmc()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--ppo-iters", type=int, default=3, help="timed DGPPO collect+update iterations (0: skip)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    local = local % ndev if ndev > 0 else local  # identity on a full node; wraps for one-GPU rehearsals
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        # RCCL over xGMI; DGPPO_DIST_BACKEND=gloo rehearses the multi-rank path with several ranks
        # sharing one GPU (RCCL refuses two ranks on one device)
        backend = os.environ.get("DGPPO_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from dgppo_fov_amd.env import make_env
    from dgppo_fov_amd.trainer.rollout import RolloutEngine

    env = make_env(ENV_ID, N_AGENTS, num_obs=N_OBS, device=dev)
    lanes = int(os.environ.get("DGPPO_BENCH_LANES", "2"))
    eng = RolloutEngine(env, B_PER_GPU, T, dev, env_offset=rank * B_PER_GPU, lanes=lanes)
    gen = torch.Generator(device=dev)
    gen.manual_seed(1000 + rank)
    eng.actions.uniform_(-1.0, 1.0, generator=gen)  # synthetic actions, resident before timing
    use_graph = not args.no_graph
    if use_graph:
        eng.capture()
    for w in range(args.warmup):
        eng.run(key=w)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for s in range(args.steps):
        eng.run(key=10_000 + s)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # ---- live kernel timing for the roofline: back-to-back step launches on the launch stream ----
    stream = torch.cuda.current_stream(dev)
    n_launch = 4 * T
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g_step = None
    cur = eng.graph_at(0)
    outs = [eng.graph_at(1), eng.graph_at(2)]

    def step_loop():  # ping-pong: step i reads buffer (i-1)&1 (graph 0 for i = 0), writes i&1
        for i in range(n_launch):
            src = cur if i == 0 else outs[(i - 1) & 1]
            env.step_into(src, eng.actions[i % T], outs[i & 1], eng.rewards[i % T], eng.costs[i % T])

    step_loop()
    torch.cuda.synchronize(dev)
    if use_graph:
        g_step = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g_step):
            step_loop()
    kern_ms = []
    for rep in range(3):
        ev0.record(stream)
        if g_step is not None:
            g_step.replay()
        else:
            step_loop()
        ev1.record(stream)
        ev1.synchronize()
        kern_ms.append(ev0.elapsed_time(ev1) / n_launch)
    step_ms = float(np.median(kern_ms))

    env_steps = args.steps * B_PER_GPU * T * world
    value = env_steps / elapsed
    bytes_per_launch = BYTES_PER_ENV_STEP * B_PER_GPU
    achieved = bytes_per_launch / (step_ms * 1e-3) / 1e9
    traffic = read_pmc_traffic()
    del eng, outs, cur, g_step
    ppo = ppo_bench(env, dev, world, rank, args.ppo_iters) if args.ppo_iters > 0 else None
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (Philox-sampled resets, uniform random actions in HBM)",
            "config": {
                "workload": f"{ENV_ID} n={N_AGENTS} obs={N_OBS} rays=32 top_k=8, {B_PER_GPU} envs/GPU, "
                            f"1 step = reset + T={T} fused env steps into the (B,T+1) rollout buffer",
                "env": ENV_ID, "num_agents": N_AGENTS, "n_obs": N_OBS, "n_env_per_gpu": B_PER_GPU, "T": T,
                "hip_graph": use_graph, "stream_lanes": lanes, "parallelism": f"dp{world} (env-sharded, no collective)",
            },
            "env_step_kernel_us": round(step_ms * 1e3, 3),
            # whole timed region (reset + T steps, 2 env slices on 2 streams) at the per-transition bytes
            "rollout_effective_hbm_gbs": round(value / world * BYTES_PER_ENV_STEP / 1e9, 1),
            "ppo_updates_per_s": None if ppo is None else ppo["updates_per_s"],
            "ppo": ppo,
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "kernel": "wv::lidar_step_wave_kernel<LIDAR,SPREAD,4,3,false>",
                "algorithmic_bytes_per_launch": bytes_per_launch,
            },
            "cpu_baseline": None if args.no_cpu_baseline or world > 1 else cpu_baseline(),
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

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
cpu_baseline: the NumPy oracle (oracle/env.py) on the host cores (one process per core), warm-up 3 and
median of 10; cpu_baseline_update: the torch-CPU fp32 network oracle (oracle/nets_t.py) on a sample of the
update's minibatch work, scaled to one update (both run before the GPU is touched).
GPU timing: `value` = env transitions / wall time of exactly K steps between barriers; the per-step
median from HIP events is reported beside it (warm-up 10, median of 50 = the defaults).
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
B_TOTAL_STRONG = 4096  # --strong: the whole job's envs (BASELINE.md strong-scaling variant)
BYTES_PER_ENV_STEP = 8856  # SURVEY.md §8(d), LidarSpread n8 O3
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def _cpu_workers() -> int:
    """Host cores to use: the process's CPU share (16 on the GPU box, whose nproc shows the whole
    machine; OMP_NUM_THREADS is set to that share there), else the affinity mask."""
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    return max(1, min(share, aff) if share > 0 else aff)


CPU_STEPS_PER_ITER, CPU_WARMUP, CPU_ITERS = 16, 3, 10  # warm-up 3, median of 10


def _cpu_env_worker(args):
    """One shard of the CPU env baseline (forked before any GPU use): NumPy oracle env steps over its
    envs, CPU_WARMUP untimed + CPU_ITERS timed iterations of CPU_STEPS_PER_ITER steps."""
    w, n_env = args
    os.environ["OMP_NUM_THREADS"] = "1"
    from oracle import env as O

    spec = O.Spec(ENV_ID, N_AGENTS, N_OBS)
    ag, gl, third = O.env_reset(spec, 1, n_env, env_offset=w * n_env)
    states = O.initial_graph(spec, ag, gl, third)["states"]
    rng = np.random.default_rng(1000 + w)
    times = []
    for it in range(CPU_WARMUP + CPU_ITERS):
        acts = rng.uniform(-1, 1, (CPU_STEPS_PER_ITER, n_env, N_AGENTS, 2)).astype(np.float32)
        t0 = time.perf_counter()
        for k in range(CPU_STEPS_PER_ITER):
            states = O.env_step(spec, states, third, acts[k])["states"]
        if it >= CPU_WARMUP:
            times.append(time.perf_counter() - t0)
    return times


def cpu_baseline():
    """The NumPy oracle (oracle/env.py, the reference's env step restated, fp32, vectorised over envs)
    on the host cores: the bench's 4096 LidarSpread n=8 envs sharded over one forked process per core
    (all host cores, warm-up 3, median of 10).  Runs BEFORE the process touches the GPU."""
    import multiprocessing as mp

    P = _cpu_workers()
    B = 4096 if P >= 8 else 1024  # the bench width on the GPU box's 16-core share
    per = [B // P + (1 if w < B % P else 0) for w in range(P)]
    with mp.get_context("fork").Pool(P) as pool:
        res = pool.map(_cpu_env_worker, list(enumerate(per)))
    # throughput = sum over shards of envs x steps / that shard's median iteration time
    value = sum(nw * CPU_STEPS_PER_ITER / float(np.median(ts)) for nw, ts in zip(per, res))
    tot = sum(sum(ts) for ts in res) / P
    return {"value": round(value, 1), "unit": "env-steps/s", "cores": P, "kind": "port", "cpu": _cpu_model(),
            "sample": f"oracle/env.py NumPy fp32, {B} LidarSpread n=8 o=3 envs sharded over {P} processes "
                      f"(1 thread each); per shard {CPU_WARMUP} warm-up + median of {CPU_ITERS} iterations of "
                      f"{CPU_STEPS_PER_ITER} env steps ({tot:.1f} s timed per process, reset excluded)"}


def cpu_baseline_update():
    """torch-CPU fp32 of the DGPPO update's minibatch work (oracle/nets_t.py: the reference's per-edge
    GraphTransformer, MLP, GRU, TanhNormal restated, every graph of the batch evaluated as one disjoint
    union graph as vmap does): update_Vl + update_Vh + update_policy forward + backward on a bounded
    sample of SAMPLE_ENVS envs x T steps, torch.set_num_threads(host cores), warm-up 3, median of 10.
    Scaled to one update = 32 minibatches x (16,384 / sample graphs) x t_sample, plus the prepass on the same
    sample (forward only: the Vl scan and Vh on the rollout and the deterministic rollout's graphs) and the
    deterministic rollout itself (actor mode + NumPy env step, T steps of the sample envs), both scaled by
    B / SAMPLE_ENVS (median of 3 after 1 warm-up)."""
    import torch as th

    from oracle import env as O
    from oracle import nets_t as R

    P = _cpu_workers()
    th.set_num_threads(P)
    SAMPLE_ENVS, L = 2, RNN_STEP
    spec = O.Spec(ENV_ID, N_AGENTS, N_OBS)
    ag, gl, third = O.env_reset(spec, 3, SAMPLE_ENVS)
    g = g0 = O.initial_graph(spec, ag, gl, third)
    rng = np.random.default_rng(2)
    seq = {k: [] for k in ("nodes", "edges", "receivers", "senders")}
    states = g["states"]
    for t in range(T):
        for k in seq:
            seq[k].append(g[k])
        g = O.env_step(spec, states, third, rng.uniform(-1, 1, (SAMPLE_ENVS, N_AGENTS, 2)).astype(np.float32))
        states = g["states"]
    graph = {k: np.stack(v, 1).reshape((SAMPLE_ENVS * T,) + v[0].shape[1:]) for k, v in seq.items()}
    G = SAMPLE_ENVS * T
    S = G // L
    n = N_AGENTS
    R.T64 = th.float32
    try:
        trees = _random_flax_trees(spec)
        acts = rng.uniform(-0.99, 0.99, (G * n, 2)).astype(np.float32)
        eps = rng.standard_normal((n, 2)).astype(np.float32)
        h_act = (rng.standard_normal((G, n, 64)) * 0.3).astype(np.float32)
        tgt_l = th.tensor(rng.standard_normal((S, L)), dtype=th.float32)
        tgt_h = th.tensor(rng.standard_normal((G, n, 2)), dtype=th.float32)
        adv = rng.standard_normal((S, L, n)).astype(np.float32)
        lp_old = rng.standard_normal((S, L, n)).astype(np.float32) - 2.0

        def one():
            pa, pl, ph = (R.to_t(x, requires_grad=True) for x in trees)
            v = R.vl_seq(pl, graph, S, L, n)
            (0.5 * (v - tgt_l) ** 2).mean().backward()
            out = R.vh(ph, graph, h_act, n)
            (0.5 * (out - tgt_h) ** 2).mean().backward()
            lp, ent = R.actor_eval_seq(pa, graph, S, L, n, acts, eps)
            R.ppo_loss(lp, lp_old, adv, ent).backward()

        def prepass_and_det():
            pa, pl, ph = (R.to_t(x) for x in trees)
            with th.no_grad():
                R.vl_seq(pl, graph, S, L, n)
                R.vh(ph, graph, h_act, n)  # the rollout's graphs
                R.vh(ph, graph, h_act, n)  # the deterministic rollout's graphs (same shapes)
                gd, h = g0, np.zeros((SAMPLE_ENVS, n, 64), np.float32)
                for t in range(T):  # the deterministic rollout: actor mode + env step
                    h2 = R.actor_carry(pa, gd, h, n)
                    mu, _ = R.policy_dist(pa, h2)
                    h = h2.numpy()
                    gd = O.env_step(spec, gd["states"], third, th.tanh(mu).numpy())

        times = []
        for it in range(CPU_WARMUP + CPU_ITERS):
            t0 = time.perf_counter()
            one()
            if it >= CPU_WARMUP:
                times.append(time.perf_counter() - t0)
        times_pd = []
        for it in range(1 + 3):
            t0 = time.perf_counter()
            prepass_and_det()
            if it >= 1:
                times_pd.append(time.perf_counter() - t0)
    finally:
        R.T64 = th.float64
    t_sample = float(np.median(times))
    t_pd = float(np.median(times_pd))
    t_update = t_sample * (PPO_BATCH / G) * (B_PER_GPU * T // PPO_BATCH) + t_pd * (B_PER_GPU / SAMPLE_ENVS)
    return {"value": round(1.0 / t_update, 6), "unit": "PPO-updates/s", "cores": P, "kind": "port",
            "cpu": _cpu_model(), "sample_ms": round(t_sample * 1e3, 2), "prepass_det_sample_ms": round(t_pd * 1e3, 2),
            "sample": f"oracle/nets_t.py torch-CPU fp32 ({P} threads): Vl + Vh + policy forward+backward on "
                      f"{SAMPLE_ENVS} envs x T={T} LidarSpread n=8 graphs ({S} rnn_step-{L} chunks), warm-up "
                      f"{CPU_WARMUP}, median of {CPU_ITERS} = {t_sample * 1e3:.1f} ms; scaled x{PPO_BATCH // G} "
                      f"to a 16,384-graph minibatch and x{B_PER_GPU * T // PPO_BATCH} minibatches per update; "
                      f"plus the prepass (Vl scan, Vh x2, forward) and the deterministic rollout (actor + env, "
                      f"{T} steps) on the same {SAMPLE_ENVS} envs = {t_pd * 1e3:.1f} ms (median of 3), "
                      f"x{B_PER_GPU // SAMPLE_ENVS}"}


def cpu_baseline_rollout():
    """The policy rollout on the host ("full rollouts with policy inference"): oracle/env.py
    NumPy fp32 env steps + the torch-CPU fp32 actor (oracle/nets_t.py: per-edge GraphTransformer GNN, MLP
    head, GRU, TanhNormal sample) on a bounded sample of ROLL_ENVS envs x ROLL_STEPS steps,
    torch.set_num_threads(host cores), warm-up 1 + median of 3 episodes-fragments.  env-steps/s."""
    import torch as th

    from oracle import env as O
    from oracle import nets_t as R

    P = _cpu_workers()
    th.set_num_threads(P)
    ROLL_ENVS, ROLL_STEPS = 256, 16
    spec = O.Spec(ENV_ID, N_AGENTS, N_OBS)
    ag, gl, third = O.env_reset(spec, 5, ROLL_ENVS)
    g0 = O.initial_graph(spec, ag, gl, third)
    rng = np.random.default_rng(3)
    R.T64 = th.float32
    try:
        pa = R.to_t(_random_flax_trees(spec)[0])

        def fragment():
            g, h = g0, np.zeros((ROLL_ENVS, N_AGENTS, 64), np.float32)
            for t in range(ROLL_STEPS):
                with th.no_grad():
                    h2 = R.actor_carry(pa, g, h, N_AGENTS)
                    mu, sd = R.policy_dist(pa, h2)
                    eps = th.as_tensor(rng.standard_normal(mu.shape), dtype=th.float32)
                    a = th.tanh(mu + sd * eps)
                    R.tanh_normal_log_prob(a, mu, sd)
                h = h2.numpy()
                g = O.env_step(spec, g["states"], third, a.numpy())
        times = []
        for it in range(1 + 3):
            t0 = time.perf_counter()
            fragment()
            if it >= 1:
                times.append(time.perf_counter() - t0)
    finally:
        R.T64 = th.float64
    t = float(np.median(times))
    return {"value": round(ROLL_ENVS * ROLL_STEPS / t, 1), "unit": "env-steps/s", "cores": P, "kind": "port",
            "cpu": _cpu_model(),
            "sample": f"oracle/env.py NumPy fp32 env steps + oracle/nets_t.py torch-CPU fp32 actor sample_action "
                      f"({P} threads) on {ROLL_ENVS} LidarSpread n=8 o=3 envs x {ROLL_STEPS} steps, warm-up 1, "
                      f"median of 3 = {t:.2f} s"}


def _random_flax_trees(spec):
    """Random-init actor / Vl / Vh parameter trees in the reference's flax layout (built on the host)."""
    from dgppo_fov_amd.algo.module.nets import ActorNet, VhNet, VlNet

    nd = spec.nd  # node features: state + 3 indicator columns (lidar_env/base.py:227-271)
    return [ActorNet(nd, N_AGENTS, "cpu", seed=6).flax(), VlNet(nd, N_AGENTS, "cpu", seed=7).flax(),
            VhNet(nd, N_AGENTS, 2, "cpu", seed=8).flax()]


def latest_profile(suffix):
    """The newest round's `profiles/rNN_<suffix>` (file name)."""
    import glob

    found = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{suffix}")))
    return os.path.basename(found[-1]) if found else suffix


def read_pmc_traffic(fn="env_step_pmc.json"):
    fn = os.path.join(ROOT, "profiles", fn)
    if os.path.exists(fn):
        try:
            return json.load(open(fn)).get("hbm_bytes_per_launch")
        except Exception:
            return None
    return None


def read_mfma_pmc():
    """Executed-MFMA utilisation from the committed PMC profile (scripts/mfma_pmc.sh): SQ_INSTS_VALU_MFMA_MOPS_F32
    x 512 per kernel family over one collect + update, against the fp32 MFMA peak."""
    import glob

    found = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_mfma_util.json")))  # the latest round's profile
    if not found:
        return None
    fn = found[-1]
    try:
        d = json.load(open(fn))
        fam = d["families"]
        gemm_t = sum(fam[k]["time_ms"] for k in ("gemm_rows", "gemm_wgrad") if k in fam)
        gemm_f = sum(fam[k]["mfma_tflop"] for k in ("gemm_rows", "gemm_wgrad") if k in fam)
        return {"source": f"profiles/{os.path.basename(fn)} (rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F32)",
                "gnn_gemm_executed_tflops": round(gemm_f / gemm_t * 1e3, 2),
                "gnn_gemm_frac_of_peak": round(gemm_f / gemm_t * 1e3 / FP32_MFMA_PEAK_TFLOPS, 4),
                "window_executed_tflops": d["total_mfma_tflops_over_window"],
                "window_frac_of_peak": round(d["total_mfma_tflops_over_window"] / FP32_MFMA_PEAK_TFLOPS, 4),
                "update_window_ms": None if "update_window_s" not in d else round(d["update_window_s"] * 1e3, 2),
                "update_mfma_tflop": d.get("update_mfma_tflop"), "update_valu_fp32_tflop": d.get("update_valu_fp32_tflop"),
                "valu_calibration": d.get("valu_calibration"), "src_sha256": d.get("src_sha256")}
    except Exception:
        return None


def source_sha256():
    """sha256 over the native sources (dgppo_fov_amd/csrc/*, include/dgppo_hip.h) in name order: the identity of
    the build a committed PMC profile measured."""
    import glob
    import hashlib

    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(ROOT, "dgppo_fov_amd", "csrc", "*"))) + [os.path.join(ROOT, "include", "dgppo_hip.h")]
    for fn in files:
        h.update(os.path.basename(fn).encode())
        h.update(open(fn, "rb").read())
    return h.hexdigest()


PPO_BATCH, RNN_STEP = 16384, 16  # BASELINE.md synthetic-input plan (batch_size, rnn_step)
# the update's algorithmic flops: dgppo_fov_amd/utils/flops.py counts the per-receiver formulation the kernels
# implement (DESIGN.md §4, §3.3 "Update flops"), not SURVEY.md §8(d)'s node-level count (22.1 TF + 2.65 TF det
# rollout at this config, 4-5x more than the kernels need); fp32 MFMA and VALU share the 157.3 TF/s peak
FP32_MFMA_PEAK_TFLOPS = 157.3


def ppo_bench(env, dev, world, rank, iters, strong=False):
    """DGPPO training iterations at the bench config: collect (policy rollout, 4096 envs x T=128 in
    one hipGraph) + update (det rollout, Vl/Vh prepass, GAE, advantages, 32 minibatches x
    [Vl, Vh, policy fwd+bwd, one grad all-reduce, clip + Adam]).  Random-init nets, synthetic envs.
    Max over ranks of the wall time between barriers."""
    from dgppo_fov_amd.algo import make_algo
    from dgppo_fov_amd.nn import kernels as K

    batch = PPO_BATCH if strong else PPO_BATCH * world  # strong: the global minibatch stays 16,384 samples
    algo = make_algo("dgppo", env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                     action_dim=env.action_dim, n_agents=N_AGENTS, batch_size=batch, rnn_step=RNN_STEP,
                     seed=0, device=dev, train_steps=1000)
    r = algo.collect(algo.params, 0, n_env=B_PER_GPU)
    algo.update(r, 0)  # warm-up: captures the deterministic-rollout graph, grows workspaces
    K.GEMM_LOG = []
    algo.update(r, 0)
    gemm_flops = sum(2.0 * M * N * Kd * b for (M, N, Kd, b, *_rest) in K.GEMM_LOG)
    K.GEMM_LOG = None
    cols, upds = [], []
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
        cols.append(t1 - t0)
        upds.append(t2 - t1)
    t = torch.tensor([cols, upds], device=dev, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)  # per iteration, the slowest rank
    t_col, t_upd = (float(x) for x in t.median(dim=1).values.tolist())
    t_upd_mean = float(t[1].mean())
    pmc = read_mfma_pmc()
    executed = None
    if pmc is not None and pmc.get("update_mfma_tflop") is not None:
        # the hardware's executed fp32 MFMA flops of one update (PMC profile of the same config: a count, independent
        # of timing) over THIS run's measured update time -- quoted only when the profile measured this tree's native
        # sources (sha256), so a stale profile fails instead of being quoted.  The profiled update window is
        # reported beside it; it runs longer than the live update because kernel tracing adds per-dispatch overhead
        # to the ~6,000 dispatches of an update.
        live = source_sha256()
        if pmc.get("src_sha256") != live:
            executed = {"status": f"not quoted: {pmc['source'].split()[0]} profiled sources {pmc.get('src_sha256')}, "
                                  f"this tree's sources are {live}"}
        elif world != 1 or strong:
            executed = {"status": "not quoted: the profile is a 1-GPU weak-scaling run"}
        else:
            ach = pmc["update_mfma_tflop"] / t_upd
            executed = {"achieved": round(ach, 2), "frac": round(ach / FP32_MFMA_PEAK_TFLOPS, 4),
                        "tflop_per_update": pmc["update_mfma_tflop"], "profile_update_ms_traced": pmc["update_window_ms"],
                        "src_sha256": live}
            if pmc.get("update_valu_fp32_tflop") is not None:
                # fp32 MFMA runs at the fp32 VALU rate on gfx950 (157.3 TF either way), so the executed fp32 work of
                # both pipes over the update time is the utilisation of the one fp32 roof
                tf = pmc["update_mfma_tflop"] + pmc["update_valu_fp32_tflop"]
                executed_fp32 = {"achieved": round(tf / t_upd, 2), "frac": round(tf / t_upd / FP32_MFMA_PEAK_TFLOPS, 4),
                                 "tflop_per_update": round(tf, 4), "mfma_tflop": pmc["update_mfma_tflop"],
                                 "valu_tflop": pmc["update_valu_fp32_tflop"],
                                 "counters": "SQ_INSTS_VALU_MFMA_MOPS_F32 x 512 + SQ_INSTS_VALU_FLOPS_FP32(_TRANS) "
                                             "calibrated on known elementwise work (valu_calibration)",
                                 "valu_calibration": pmc.get("valu_calibration")}
                executed["executed_fp32"] = executed_fp32
    from dgppo_fov_amd.utils.flops import update_flops

    fl = update_flops(algo, env, B_PER_GPU, T)  # per rank; the deterministic rollout's actor inference included
    upd_tf = fl["total"] * world / 1e12
    return {"updates_per_s": round(1.0 / t_upd, 4), "update_ms": round(t_upd * 1e3, 2),
            "update_ms_mean": round(t_upd_mean * 1e3, 2), "timing": f"median of {iters} iterations after 2 warm-up updates",
            "update_roofline": {"bound": "mfma", "algorithmic_tflop": round(upd_tf, 2),
                                "achieved": round(upd_tf / t_upd, 2), "peak": FP32_MFMA_PEAK_TFLOPS * world,
                                "unit": "TFLOP/s", "frac": round(upd_tf / t_upd / (FP32_MFMA_PEAK_TFLOPS * world), 4),
                                "frac_kind": "algorithmic: the per-receiver formulation the kernels implement "
                                             "(dgppo_fov_amd/utils/flops.py, DESIGN.md 3.3); the hardware's executed "
                                             "work is executed_mfma / executed_fp32",
                                "flops_source": "utils/flops.py update_flops: " + ", ".join(
                                    f"{k} {v / 1e12:.3f} TF" for k, v in fl["parts"].items()),
                                "per_graph_fwd_mflop": fl["per_graph_fwd_mflop"],
                                "survey_8d_node_level_tflop": round((22.1 + 2.65) * (B_PER_GPU / 4096) * world, 2),
                                "executed_mfma": executed},
            "collect_ms": round(t_col * 1e3, 2),
            "collect_env_steps_per_s": round(B_PER_GPU * T * world / t_col, 1),
            "iters": iters, "batch_size": batch, "rnn_step": RNN_STEP, "epoch_ppo": 1,
            "minibatches": B_PER_GPU * T * world // batch,
            "gemm_tflop_per_update": round(gemm_flops / 1e12, 3),
            "gemm_tflops_over_update": round(gemm_flops / t_upd / 1e12, 3), "fp32_mfma_peak_tflops": 157.3,
            "mfma_pmc": pmc}


def _free_port() -> int:
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int) -> int:
    """`bench.py --gpus N` run directly (no torchrun): start N fresh child processes of this script, one per
    GPU, with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set, exactly as
    `torch.distributed.run --nproc-per-node N` would; rank 0 prints the JSON line.  This parent never
    touches the GPU (no HIP call before or after the children), and if a rank fails the others are
    terminated.  Returns the first non-zero exit code (0 when every rank succeeded)."""
    import subprocess

    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    while procs:
        for p in list(procs):
            code = p.poll()
            if code is None:
                continue
            procs.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in procs:
                    q.terminate()
        time.sleep(0.2)
    return rc


def main():
    global B_PER_GPU
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)  # warm-up 10, median of 50
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling: 4096 envs (and the 16,384-sample PPO batch) in total, split over the ranks")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--ppo-iters", type=int, default=10, help="timed DGPPO collect+update iterations (0: skip)")
    ap.add_argument("--print-rank-env", action="store_true", help=argparse.SUPPRESS)  # launcher test (CPU only)
    args = ap.parse_args()

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(env_world or "1")
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch one rank per GPU "
                 f"(torch.distributed.run --nproc-per-node {args.gpus}) or drop WORLD_SIZE")
    rank = int(os.environ.get("RANK", "0"))
    if args.print_rank_env:  # tests/test_bench_cpu.py: what each launched rank sees, before any GPU use
        print(json.dumps({k: os.environ.get(k) for k in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR",
                                                          "MASTER_PORT")}), flush=True)
        return
    if args.strong:
        if B_TOTAL_STRONG % world:
            sys.exit(f"bench.py --strong: {B_TOTAL_STRONG} envs do not split over {world} ranks")
        B_PER_GPU = B_TOTAL_STRONG // world
    # CPU baselines first: forked workers must never inherit an initialised GPU context
    cpu_env = cpu_upd = cpu_roll = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu_env = cpu_baseline()
        cpu_roll = cpu_baseline_rollout()
        cpu_upd = cpu_baseline_update() if args.ppo_iters > 0 else None

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
    lanes = int(os.environ.get("DGPPO_BENCH_LANES", "1"))  # 1: states-only reset + ONE persistent rollout launch
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
    stream = torch.cuda.current_stream(dev)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for s in range(args.steps):
        evs[s].record(stream)
        eng.run(key=10_000 + s)
    evs[-1].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    step_ms_median = float(np.median([evs[i].elapsed_time(evs[i + 1]) for i in range(args.steps)]))

    # ---- live kernel timing for the roofline (HIP events on the launch stream) ----
    stream = torch.cuda.current_stream(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # (a) the dominant kernel: the persistent rollout kernel alone (T steps from the loaded graph 0)
    roll_ms = None
    if eng.fused and lanes == 1:
        # back-to-back launches (a captured graph of 4 when graphs are on), so no host dispatch gap sits
        # between the events: the per-launch figure is the kernel's own duration, as rocprof reports it
        def roll4():
            for _ in range(4):
                env.rollout_into(eng.buf, eng.obstacles, eng.actions, eng.rewards, eng.costs, rebuild_first=False)

        roll4()
        torch.cuda.synchronize(dev)
        g_roll = None
        if use_graph:
            g_roll = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g_roll):
                roll4()
        rms = []
        for rep in range(6):
            ev0.record(stream)
            if g_roll is not None:
                g_roll.replay()
            else:
                roll4()
            ev1.record(stream)
            ev1.synchronize()
            if rep:
                rms.append(ev0.elapsed_time(ev1) / 4)
        roll_ms = float(np.median(rms))
    # (b) the per-step kernel (policy rollouts use it): back-to-back step launches in a hipGraph
    n_launch = 4 * T
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
    for rep in range(5):
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
    if roll_ms is not None:  # T transitions per launch
        bytes_per_launch = BYTES_PER_ENV_STEP * B_PER_GPU * T
        achieved = bytes_per_launch / (roll_ms * 1e-3) / 1e9
        kname = "wv::lidar_rollout_wave_kernel<LIDAR,SPREAD,4,3> (persistent: T=128 steps per launch)"
    else:
        bytes_per_launch = BYTES_PER_ENV_STEP * B_PER_GPU
        achieved = bytes_per_launch / (step_ms * 1e-3) / 1e9
        kname = "wv::lidar_step_wave_kernel<LIDAR,SPREAD,4,3,false>"
    step_achieved = BYTES_PER_ENV_STEP * B_PER_GPU / (step_ms * 1e-3) / 1e9
    traffic = read_pmc_traffic(latest_profile("env_rollout_pmc.json") if roll_ms is not None else "env_step_pmc.json")
    fused = eng.fused and lanes == 1
    del eng, outs, cur, g_step
    ppo = ppo_bench(env, dev, world, rank, args.ppo_iters, strong=args.strong) if args.ppo_iters > 0 else None
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "ms_per_step_median": round(step_ms_median, 4),  # HIP events around each step, rank 0
            "higher_is_better": True,
            "scaling": "strong" if args.strong else "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (Philox-sampled resets, uniform random actions in HBM)",
            "config": {
                "workload": f"{ENV_ID} n={N_AGENTS} obs={N_OBS} rays=32 top_k=8, {B_PER_GPU} envs/GPU"
                            f"{f' ({B_PER_GPU * world} in total, strong scaling)' if args.strong else ''}, "
                            f"1 step = reset + T={T} fused env steps into the (B,T+1) rollout buffer",
                "env": ENV_ID, "num_agents": N_AGENTS, "n_obs": N_OBS, "n_env_per_gpu": B_PER_GPU, "T": T,
                "hip_graph": use_graph, "stream_lanes": lanes, "persistent_rollout": fused,
                "parallelism": f"dp{world} (env-sharded, no collective)",
            },
            "env_step_kernel_us": round(step_ms * 1e3, 3),
            "env_step_kernel_gbs": round(step_achieved, 1),  # the per-step kernel the policy rollouts launch
            "env_rollout_kernel_us": None if roll_ms is None else round(roll_ms * 1e3, 2),
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
                "kernel": kname,
                "algorithmic_bytes_per_launch": bytes_per_launch,
            },
            "cpu_baseline": cpu_env,
            "cpu_baseline_update": cpu_upd,
            "cpu_baseline_rollout": cpu_roll,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

"""DGPPO (dgppo/algo/dgppo.py:25-321 + its bases informarl_lagr.py / informarl.py) on MI355X.

Same public surface as the reference Algorithm (dgppo/algo/base.py:10-99): `params`, `config`,
`init_rnn_state`, `act`, `step`, `collect`, `update`, `save`, `load`.  Every numeric step runs in
libdgppo_hip.so:

  collect      RolloutEngine (env reset + T x [actor step + fused env step]) in one hipGraph
  update       det rollout (get_action) -> Vl scan (prepass) -> Vh on both rollouts ->
               Dec-OCP GAE -> DGPPO advantages -> per minibatch: update_Vl, update_Vh,
               update_policy (fwd+bwd through the GNN/MLP/GRU kernels, losses, global-norm clip,
               finite check, Adam), dgppo.py:136-321 / informarl.py:357-457.

Multi-GPU (torch.distributed over RCCL): each rank owns a shard of the envs; the minibatch is the
k-th env chunk of every rank's local shuffle; the three nets' gradients live in ONE flat buffer
and are all-reduced (mean) once per minibatch before clip + Adam, so replicas stay identical.
"""
from __future__ import annotations

import math
import os
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

from ..env.base import MultiAgentEnv
from ..nn import kernels as K
from ..nn.layers import GraphBatch
from ..trainer.data import Rollout
from ..trainer.rollout import RolloutEngine
from .module.nets import ActorNet, VhNet, VlNet


def minibatch_plan(n_env_local: int, T: int, world: int, batch_size: int, rng: np.random.Generator):
    """Env-index minibatches of one PPO epoch for this rank (dgppo.py:155-159 sharded): the reference
    permutes all B envs and splits them into B / (batch_size / T) minibatches; with p ranks each rank
    permutes its own B/p envs and minibatch k is the k-th chunk of every rank's permutation (same
    global minibatch size, rank-local shuffle).  Returns a list of index arrays."""
    mb_envs_global = batch_size // T
    n_mb = (n_env_local * world) // mb_envs_global if mb_envs_global >= 1 else 0
    if n_mb < 1 or n_env_local % n_mb != 0:  # jnp.array(jnp.array_split(...)) needs equal chunks
        raise ValueError(f"{n_mb} minibatches (batch_size {batch_size}, T {T}) do not split the "
                         f"{n_env_local} envs of a rank evenly")
    idx = np.arange(n_env_local)
    rng.shuffle(idx)
    return np.array_split(idx, n_mb)


def allreduce_mean_(t: torch.Tensor, world: int, force: bool = False):
    """In-place mean over ranks (one collective: SUM then scale; RCCL on GPUs, gloo on CPU).  force: run the
    collective on a one-rank group too (DGPPO_FORCE_ALLREDUCE, the RCCL path's world-size-1 test)."""
    if world > 1 or force:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        t.mul_(1.0 / world)
    return t


# graphs per prepass chunk (the Vl scan / Vh passes over the whole rollout run env chunks of this many graphs)
PREPASS_GRAPHS = int(os.environ.get("DGPPO_PREPASS_GRAPHS", 65536))


def PHASE_EVENTS() -> bool:
    """Timing knob: HIP-event split of update() into prepass / GAE + advantages / minibatches (no synchronisation)."""
    return os.environ.get("DGPPO_PHASE_EVENTS", "0") == "1"


def ADAM_MULTI() -> bool:
    """The three nets' clip + Adam steps in two launches (dgppo_adam_multi) instead of four per net (default on)."""
    return os.environ.get("DGPPO_ADAM_MULTI", "1") == "1"


def DEFER_WGRAD() -> bool:
    """Each net's weight-gradient GEMMs deferred to the end of its backward and launched as one grouped kernel
    (K.defer_wgrad, dgppo_gemm_wgrad_grouped): bit-identical, fewer launches (DGPPO_DEFER_WGRAD=0: one launch pair
    per GEMM)."""
    return os.environ.get("DGPPO_DEFER_WGRAD", "1") == "1"


def FORCE_SAFE() -> bool:
    """Learning-dynamics ablation (scripts/learn_ablate.sh): treat every sample as inside the safe set."""
    return os.environ.get("DGPPO_DEBUG_FORCE_SAFE", "0") == "1"


class _Phases:
    """Host wall-clock per update phase (synchronising) when DGPPO_PROFILE=1; no-op otherwise."""

    def __init__(self, device):
        self.on = os.environ.get("DGPPO_PROFILE", "0") == "1"
        self.device = device
        self.acc = {}
        self.t = None

    def mark(self, name=None):
        if not self.on:
            return
        import time
        torch.cuda.synchronize(self.device)
        now = time.perf_counter()
        if name is not None and self.t is not None:
            self.acc[name] = self.acc.get(name, 0.0) + now - self.t
        self.t = now

    def report(self):
        if self.on and self.acc:
            tot = sum(self.acc.values())
            print("DGPPO update phases (ms): " + ", ".join(f"{k} {1e3 * v:.1f}" for k, v in self.acc.items()) +
                  f" | total {1e3 * tot:.1f}", flush=True)


class _Opt:
    """optax.apply_if_finite(optax.adam(lr), 1e6) state + compute_norm_and_clip for one flat buffer."""

    def __init__(self, ps, lr, max_norm, device):
        self.ps, self.lr, self.max_norm = ps, lr, max_norm
        self.m = torch.zeros_like(ps.flat)
        self.v = torch.zeros_like(ps.flat)
        self.state = torch.zeros(3, dtype=torch.float32, device=device)  # [norm, non-finite, count]

    def step(self):
        K.grad_norm(self.ps.grad, self.state)
        K.adam(self.ps.flat, self.ps.grad, self.m, self.v, self.state, self.lr, max_norm=self.max_norm)


class DGPPO:
    VH_NET = VhNet  # the cost critic's network class (InforMARL-Lagr: VhGlobalNet)

    def __init__(self, env: MultiAgentEnv, node_dim: int, edge_dim: int, state_dim: int, action_dim: int,
                 n_agents: int, actor_gnn_layers: int = 2, Vl_gnn_layers: int = 2, Vh_gnn_layers: int = 1,
                 gamma: float = 0.99, lr_actor: float = 3e-4, lr_Vl: float = 1e-3, lr_Vh: float = 1e-3,
                 batch_size: int = 8192, epoch_ppo: int = 1, clip_eps: float = 0.25, gae_lambda: float = 0.95,
                 coef_ent: float = 1e-2, max_grad_norm: float = 2.0, seed: int = 0, use_rnn: bool = True,
                 rnn_layers: int = 1, rnn_step: int = 16, use_lstm: bool = False, alpha: float = 10.0,
                 cbf_eps: float = 1e-2, cbf_weight: float = 1.0, train_steps: int = int(1e5),
                 cbf_schedule: bool = True, device=None, **kwargs):
        if rnn_layers < 1:
            raise ValueError(f"rnn_layers {rnn_layers} < 1")
        self._env = env
        self.device = torch.device(device) if device is not None else env.device
        self._node_dim, self._edge_dim, self._action_dim, self._n_agents = node_dim, edge_dim, action_dim, n_agents
        self.actor_gnn_layers, self.Vl_gnn_layers, self.Vh_gnn_layers = actor_gnn_layers, Vl_gnn_layers, Vh_gnn_layers
        self.gamma, self.lr_actor, self.lr_Vl, self.lr_Vh = gamma, lr_actor, lr_Vl, lr_Vh
        self.batch_size, self.epoch_ppo, self.clip_eps, self.gae_lambda = batch_size, epoch_ppo, clip_eps, gae_lambda
        self.coef_ent, self.max_grad_norm, self.seed = coef_ent, max_grad_norm, seed
        self.use_rnn, self.rnn_layers, self.rnn_step, self.use_lstm = use_rnn, rnn_layers, rnn_step, use_lstm
        self.alpha, self.cbf_eps, self.cbf_weight, self.cbf_schedule = alpha, cbf_eps, cbf_weight, cbf_schedule
        self.train_steps = int(train_steps)
        self.world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        self.rank = dist.get_rank() if self.world > 1 else 0
        # the gradient / safe-data collectives run when there are several ranks, or on a one-rank process group when
        # DGPPO_FORCE_ALLREDUCE=1 (tests/test_distributed_gpu.py: RCCL's code path exercised on one GPU)
        self._reduce = self.world > 1 or (os.environ.get("DGPPO_FORCE_ALLREDUCE", "0") == "1" and dist.is_available()
                                          and dist.is_initialized())

        dev = self.device
        # RNN(GRUCell | LSTMCell, rnn_layers) or none (--no-rnn / --use-lstm / --rnn-layers, nn/rnn.py:10-30)
        rk = dict(rnn="none" if not use_rnn else ("lstm" if use_lstm else "gru"), rnn_layers=rnn_layers)
        self.actor = ActorNet(node_dim, n_agents, dev, seed=seed * 3 + 0, gnn_layers=actor_gnn_layers,
                              action_dim=action_dim, edge_dim=edge_dim, **rk)
        self.Vl = VlNet(node_dim, n_agents, dev, seed=seed * 3 + 1, gnn_layers=Vl_gnn_layers, edge_dim=edge_dim, **rk)
        self.Vh = self.VH_NET(node_dim, n_agents, env.n_cost, dev, seed=seed * 3 + 2, gnn_layers=Vh_gnn_layers,
                              edge_dim=edge_dim, **rk)
        self.n_carries = self.actor.gru.carries
        # one flat gradient buffer for the three nets (one all-reduce per minibatch)
        sizes = [self.Vl.ps.size, self.Vh.ps.size, self.actor.ps.size]
        self.grad_flat = torch.zeros(sum(sizes), dtype=torch.float32, device=dev)
        off = 0
        for net, sz in zip((self.Vl, self.Vh, self.actor), sizes):
            net.ps.grad = self.grad_flat[off:off + sz]
            net.ps.build_views()
            off += sz
        self.opt = {"Vl": _Opt(self.Vl.ps, lr_Vl, max_grad_norm, dev), "Vh": _Opt(self.Vh.ps, lr_Vh, max_grad_norm, dev),
                    "policy": _Opt(self.actor.ps, lr_actor, max_grad_norm, dev)}
        # the reference draws the entropy's tanh-Jacobian sample ONCE at trace time with a fixed key,
        # identical for every vmapped env/step (distribution.py:37-43); here: a fixed (n, A) draw
        self.entropy_eps = torch.from_numpy(
            np.random.default_rng(10_000 + seed).standard_normal((n_agents, action_dim)).astype(np.float32)).to(dev)
        self.init_rnn_state = torch.zeros((rnn_layers, n_agents, self.n_carries, 64), device=dev)
        self.init_Vl_rnn_state = torch.zeros((rnn_layers, 1, self.n_carries, 64), device=dev)
        self._engines = {}
        self._capturing = False
        self._flat_reduce = False  # one flat gradient all-reduce per minibatch (the minibatch-graph path), not buckets
        self.trace: Optional[dict] = None  # set to {} to record update intermediates (parity tests)
        self.key = np.random.default_rng(seed)
        self.np_rng = np.random.default_rng(seed)

    # ---- reference properties ------------------------------------------------------------------
    @property
    def node_dim(self):
        return self._node_dim

    @property
    def edge_dim(self):
        return self._edge_dim

    @property
    def action_dim(self):
        return self._action_dim

    @property
    def n_agents(self):
        return self._n_agents

    @property
    def config(self) -> dict:
        return {
            "cost_weight": 0.0, "actor_gnn_layers": self.actor_gnn_layers, "Vl_gnn_layers": self.Vl_gnn_layers,
            "gamma": self.gamma, "lr_actor": self.lr_actor, "lr_Vl": self.lr_Vl, "batch_size": self.batch_size,
            "epoch_ppo": self.epoch_ppo, "clip_eps": self.clip_eps, "gae_lambda": self.gae_lambda,
            "coef_ent": self.coef_ent, "max_grad_norm": self.max_grad_norm, "seed": self.seed,
            "use_rnn": self.use_rnn, "rnn_layers": self.rnn_layers, "rnn_step": self.rnn_step,
            "use_lstm": self.use_lstm, "cost_schedule": False, "lr_Vh": self.lr_Vh,
            "Vh_gnn_layers": self.Vh_gnn_layers, "alpha": self.alpha, "cbf_eps": self.cbf_eps,
            "cbf_weight": self.cbf_weight, "cbf_schedule": self.cbf_schedule,
        }

    @property
    def params(self) -> dict:
        return {"policy": self.actor.ps.flat, "Vl": self.Vl.ps.flat, "Vh": self.Vh.ps.flat}

    def cbf_weight_at(self, step: int) -> float:
        """optax.piecewise_constant_schedule(cbf_weight, {0.5 T: 2, 0.75 T: 2}) (dgppo.py:73-80)."""
        w = self.cbf_weight
        if not self.cbf_schedule:
            return w
        if step >= int(self.train_steps * 0.5):
            w *= 2
        if step >= int(self.train_steps * 0.75):
            w *= 2
        return w

    def _check_params(self, params):
        """The kernels read the nets' own parameter buffers: `params` must be None or this algorithm's
        `params` (the same flat tensors), never a foreign parameter set."""
        if params is not None:
            mine = self.params
            assert set(params) == set(mine) and all(params[k] is mine[k] for k in mine), \
                "params must be this algorithm's own parameter buffers (self.params)"

    # ---- acting ----------------------------------------------------------------------------------
    def _gb(self, graph) -> GraphBatch:
        return GraphBatch.from_graph(graph, self._env)

    @staticmethod
    def _rows(rs: torch.Tensor) -> torch.Tensor:
        """Reference carry layout (..., rnn_layers, n, carries, 64) -> the kernels' agent-major rows (..., n, W)
        (a view of the rollout engine's (T+1, B, n, W) buffer)."""
        return rs.movedim(-3, -4).flatten(-3)

    def _unrows(self, h: torch.Tensor) -> torch.Tensor:
        """(..., n, W) carry rows -> the reference layout (..., rnn_layers, n, carries, 64)."""
        return h.unflatten(-1, (self.rnn_layers, self.n_carries, 64)).movedim(-4, -3)

    def act(self, graph, rnn_state: torch.Tensor, params=None):
        """get_action for a batch of graphs: rnn_state (B, rnn_layers, n, carries, 64) -> (action (B, n, A), rnn)."""
        self._check_params(params)
        g = self._gb(graph)
        B, n = g.G, self._n_agents
        h = self._rows(rnn_state).reshape(B * n, -1).contiguous()
        a, _, h2 = self.actor.act(g, h, 0)
        return a.view(B, n, -1), self._unrows(h2.view(B, n, -1))

    def step(self, graph, rnn_state: torch.Tensor, key: int, params=None):
        """sample_action: (action, log_pi (B, n), rnn)."""
        g = self._gb(graph)
        B, n = g.G, self._n_agents
        noise = torch.empty((B * n, self._action_dim), device=self.device)
        K.normal_(noise, seed=int(key))
        a, lp, h2 = self.actor.act(g, self._rows(rnn_state).reshape(B * n, -1).contiguous(), 1, noise=noise)
        return a.view(B, n, -1), lp.view(B, n), self._unrows(h2.view(B, n, -1))

    def _rollout_lanes(self, n_env: int) -> int:
        """Env slices on separate streams (RolloutEngine lanes): DGPPO_ROLLOUT_LANES when the slices are
        whole (the engine itself keeps one stream where the fused policy step does not cover the env)."""
        lanes = int(os.environ.get("DGPPO_ROLLOUT_LANES", "1"))
        return 1 if lanes <= 1 or n_env % lanes or self.device.type != "cuda" else lanes

    def _engine(self, n_env: int, mode: int) -> RolloutEngine:
        k = (n_env, mode)
        if k not in self._engines:
            eng = RolloutEngine(self._env, n_env, self._env.max_episode_steps, self.device,
                                env_offset=self.rank * n_env, actor=self.actor, mode=mode,
                                lanes=self._rollout_lanes(n_env))
            if os.environ.get("DGPPO_NO_GRAPH", "0") != "1":
                eng.capture()
            self._engines[k] = eng
        return self._engines[k]

    def collect(self, params, key, n_env: Optional[int] = None) -> Rollout:
        """jit(vmap(rollout_fn))(params, keys): `key` is an int seed (or a sequence whose length is n_env).

        The returned Rollout is a set of VIEWS into the buffers of a RolloutEngine cached per n_env:
        the next collect() with the same n_env overwrites it in place (the reference returns fresh
        arrays).  Clone the fields to keep a rollout across collects."""
        self._check_params(params)
        if n_env is None:
            n_env = len(key) if hasattr(key, "__len__") else 128
        seed = int(np.asarray(key).reshape(-1)[0]) if hasattr(key, "__len__") else int(key)
        return self._engine(n_env, RolloutEngine.MODE_SAMPLE).run(seed)

    def det_rollout(self, n_env: int, key: int) -> Rollout:
        """test_rollout with the deterministic policy; the same aliasing as collect() applies."""
        return self._engine(n_env, RolloutEngine.MODE_DET).run(key)

    # ---- update ------------------------------------------------------------------------------
    def _env_ids(self, batches):
        """Every minibatch's env ids in ONE host-to-device copy (a per-minibatch copy from pageable memory
        synchronises the stream and stalls the launch pipeline); yields (len(bi),) device views."""
        flat = torch.as_tensor(np.concatenate(batches).astype(np.int64), device=self.device)
        off = 0
        for bi in batches:
            yield flat[off:off + len(bi)]
            off += len(bi)

    @staticmethod
    def _gather(envs: torch.Tensor, *fields):
        """Contiguous (len(envs), T, ...) copies of (B, T, ...) rollout fields for the selected envs, one
        torch.ops.dgppo.gather_env_steps launch per 8 fields (the minibatch's x[idx])."""
        out = [torch.empty((envs.shape[0],) + tuple(f.shape[1:]), dtype=f.dtype, device=f.device) for f in fields]
        for i in range(0, len(fields), 8):
            torch.ops.dgppo.gather_env_steps(list(fields[i:i + 8]), out[i:i + 8], envs)
        return out

    def _graph_batch(self, nodes, edges, recv, send) -> GraphBatch:
        Be, T = nodes.shape[:2]
        return GraphBatch(nodes.view(Be * T, *nodes.shape[2:]), edges.view(Be * T, *edges.shape[2:]),
                          recv.view(Be * T, -1), send.view(Be * T, -1), self._n_agents,
                          self._env.agent_candidates(self.device), raw_cols=self._env.nonagent_feature_cols)

    def _graphs(self, graph, envs) -> GraphBatch:
        """(Be, T, ...) graphs of the selected envs, env-major -> contiguous GraphBatch."""
        if not isinstance(envs, slice):
            return self._graph_batch(*self._gather(envs, graph.nodes, graph.edges, graph.receivers, graph.senders))
        sel = lambda x: x[envs]  # noqa: E731
        nodes, edges = sel(graph.nodes).contiguous(), sel(graph.edges).contiguous()
        recv, send = sel(graph.receivers).contiguous(), sel(graph.senders).contiguous()
        Be, T = nodes.shape[:2]
        return GraphBatch(nodes.view(Be * T, *nodes.shape[2:]), edges.view(Be * T, *edges.shape[2:]),
                          recv.view(Be * T, -1), send.view(Be * T, -1), self._n_agents,
                          self._env.agent_candidates(self.device), raw_cols=self._env.nonagent_feature_cols)

    def _last_graph(self, next_graph, envs=slice(None)) -> GraphBatch:
        ng = next_graph
        return GraphBatch(ng.nodes[envs, -1], ng.edges[envs, -1], ng.receivers[envs, -1], ng.senders[envs, -1],
                          self._n_agents, self._env.agent_candidates(self.device),
                          raw_cols=self._env.nonagent_feature_cols)

    def _vl_all(self, rollout: Rollout, chunk: int) -> torch.Tensor:
        """scan_Vl over every env's whole episode from the zero carry, plus the final Vl at next_graph[:, -1]
        from the scan's last carry (final_Vl_fn_, dgppo.py:203-216): (B, T+1)."""
        B, T = rollout.rewards.shape
        Vl = torch.empty((B, T + 1), device=self.device)
        hT_all = torch.empty((B, self.Vl.carry_width), device=self.device)
        tm = self._time_major(rollout, self._rows) if hasattr(self.Vl, "graph_means") else None
        if tm is not None:
            # the GNN + agent mean over the time-major graphs in place (whole time steps per chunk; graphs are
            # independent), then head + GRU scan per env sequence from the (B, T, 64) means: bit-identical to
            # env-chunked graph copies, without copying the graphs
            (nodes, edges, recv, send), _ = tm
            zm = torch.empty((T, B, 64), device=self.device)
            tc = max(1, (chunk * T) // B)
            for t0 in range(0, T, tc):
                t1 = min(T, t0 + tc)
                G = (t1 - t0) * B
                g = GraphBatch(nodes[t0:t1].reshape(G, *nodes.shape[2:]), edges[t0:t1].reshape(G, *edges.shape[2:]),
                               recv[t0:t1].reshape(G, -1), send[t0:t1].reshape(G, -1), self._n_agents,
                               self._env.agent_candidates(self.device), raw_cols=self._env.nonagent_feature_cols)
                self.Vl.graph_means(g, out=zm[t0:t1].view(G, 64))
            zm_env = zm.transpose(0, 1).contiguous()  # (B, T, 64): rows e * T + t
            # head + GRU scan of every env in ONE pass (rows independent: bit-identical to env chunks); chunks of
            # 512 envs left the scan's 128 dependent steps on 32 workgroups, one chunk after another
            v, hT, _ = self.Vl.seq_fwd(None, B, T, keep_cache=False, zm=zm_env.view(-1, 64))
            Vl[:, :T].copy_(v)
            hT_all.copy_(hT)
        for e0 in range(0, B, chunk) if tm is None else ():
            e1 = min(B, e0 + chunk)
            g = self._graphs(rollout.graph, slice(e0, e1))
            v, hT, _ = self.Vl.seq_fwd(g, e1 - e0, T, keep_cache=False)
            Vl[e0:e1, :T].copy_(v)
            hT_all[e0:e1].copy_(hT)
        # the final values of every env in one pass (rows are independent: identical to per-chunk passes)
        vf, _, _ = self.Vl.seq_fwd(self._last_graph(rollout.next_graph), B, 1, h0=hT_all, keep_cache=False)
        Vl[:, T].copy_(vf[:, 0])
        return Vl

    @staticmethod
    def _time_major(rollout: Rollout, rows_fn):
        """(T, B, ...) contiguous views of the rollout's graph fields and carry rows when the Rollout is the
        RolloutEngine's (B, T) view of its time-major buffers (else None): passes whose graphs are independent
        (Vh: one GRU step per graph) then read the buffers in place instead of copying env chunks."""
        g = rollout.graph
        f = [x.transpose(0, 1) for x in (g.nodes, g.edges, g.receivers, g.senders)]
        h = rows_fn(rollout.rnn_states).transpose(0, 1)
        return (f, h) if all(x.is_contiguous() for x in f + [h]) else None

    def _vh_all(self, rollout: Rollout, chunk: int):
        """Vh on every (env, t) graph with the stored actor carries, plus the final Vh (dgppo.py:218-228).  Graphs
        are independent here, so the time-major rollout buffers are read in place, whole time steps at a time
        (bit-identical to env chunks: no reduction crosses graphs)."""
        B, T, n = rollout.rewards.shape[0], rollout.rewards.shape[1], self._n_agents
        out = torch.empty((B, T + 1, n, self._env.n_cost), device=self.device)
        tm = self._time_major(rollout, self._rows)
        if tm is not None:
            (nodes, edges, recv, send), hrows = tm
            tc = max(1, (chunk * T) // B)
            for t0 in range(0, T, tc):
                t1 = min(T, t0 + tc)
                G = (t1 - t0) * B
                g = GraphBatch(nodes[t0:t1].reshape(G, *nodes.shape[2:]), edges[t0:t1].reshape(G, *edges.shape[2:]),
                               recv[t0:t1].reshape(G, -1), send[t0:t1].reshape(G, -1), n,
                               self._env.agent_candidates(self.device), raw_cols=self._env.nonagent_feature_cols)
                v, _ = self.Vh.fwd(g, hrows[t0:t1].reshape(G * n, -1), keep_cache=False)
                out[:, t0:t1].copy_(v.view(t1 - t0, B, n, -1).transpose(0, 1))
        for e0 in range(0, B, chunk) if tm is None else ():
            e1 = min(B, e0 + chunk)
            g = self._graphs(rollout.graph, slice(e0, e1))
            h = self._rows(rollout.rnn_states[e0:e1]).reshape((e1 - e0) * T * n, -1).contiguous()
            v, _ = self.Vh.fwd(g, h, keep_cache=False)
            out[e0:e1, :T].copy_(v.view(e1 - e0, T, n, -1))
        # final, every env in one pass: act on next_graph[-1] from rnn_states[-1], then Vh with that carry
        gl = self._last_graph(rollout.next_graph)
        h_last = self._rows(rollout.rnn_states[:, -1]).reshape(B * n, -1).contiguous()
        _, _, h2 = self.actor.act(gl, h_last, 0)
        vf, _ = self.Vh.fwd(gl, h2, keep_cache=False)
        out[:, T].copy_(vf.view(B, n, -1))
        return out

    def _allreduce_grads(self):
        allreduce_mean_(self.grad_flat, self.world, self._reduce)

    def _start_reduce(self, net, pending: list):
        """Start the (sum) all-reduce of one net's gradient bucket as soon as its backward is done, so it
        travels over xGMI (RCCL's stream) while the next net's forward / backward runs; `_finish_reduce`
        waits for every bucket and scales by 1/world before clip + Adam (same result as one flat
        all-reduce: each bucket is reduced exactly once).  Not while a minibatch graph is being captured: the
        graph path all-reduces the whole gradient buffer eagerly between its two replays."""
        if self._reduce and not self._capturing and not self._flat_reduce:
            pending.append(dist.all_reduce(net.ps.grad, op=dist.ReduceOp.SUM, async_op=True))

    def _finish_reduce(self, pending: list):
        if self._reduce and not self._capturing:
            if self._flat_reduce:  # the graph path's eager first minibatch: the same flat all-reduce as its replays
                self._allreduce_grads()
                return
            for w in pending:
                w.wait()
            pending.clear()
            self.grad_flat.mul_(1.0 / self.world)

    def _aux_streams(self, k: int):
        """k auxiliary HIP streams for the update's independent passes (None when DGPPO_STREAMS=0 or
        when DGPPO_PROFILE phase timing is on, which synchronises between passes)."""
        if k <= 0 or os.environ.get("DGPPO_STREAMS", "1") == "0" or os.environ.get("DGPPO_PROFILE", "0") == "1":
            return None
        aux = getattr(self, "_aux", None)
        if aux is None or len(aux) < k:
            aux = self._aux = [torch.cuda.Stream(self.device) for _ in range(k)]
        return aux[:k]

    def _parallel(self, jobs):
        """Run independent closures concurrently and return their results: job 0 on the current stream,
        job i > 0 on auxiliary stream i - 1.  Every auxiliary stream first waits for all work enqueued so
        far and the current stream then waits for every auxiliary stream, so results are used, and
        buffers freed, only after the producing stream's work.  Each job's kernels keep their order, so
        the results are bit-identical to running the jobs one after another."""
        aux = self._aux_streams(len(jobs) - 1)
        if aux is None:
            return [job() for job in jobs]
        main = torch.cuda.current_stream(self.device)
        for st in aux:
            st.wait_stream(main)
        out = [None] * len(jobs)
        for k, job in enumerate(jobs[1:]):
            with torch.cuda.stream(aux[k]):
                out[k + 1] = job()
        out[0] = jobs[0]()
        for st in aux:
            main.wait_stream(st)
        return out

    def _buf(self, name: str, shape) -> torch.Tensor:
        """Update scratch that keeps its address from update to update (the captured minibatch graph reads it)."""
        bufs = self.__dict__.setdefault("_bufs", {})
        t = bufs.get(name)
        if t is None or tuple(t.shape) != tuple(shape):
            t = bufs[name] = torch.empty(shape, device=self.device)
        return t

    # minibatches of at most this many samples replay from hipGraphs by default (DGPPO_UPDATE_GRAPH=1|0 forces it):
    # a 2048-sample minibatch (config 4's 8-GPU strong share) is launch-bound, ~190 launches on three streams
    GRAPH_MAX_SAMPLES = int(os.environ.get("DGPPO_UPDATE_GRAPH_MAX", 8192))

    def _mb_graph_ok(self, batches, ph, T) -> bool:
        """Replay the minibatch step from captured hipGraphs: no parity trace, no phase timing, equal minibatch
        sizes, concurrent streams on; by default for small minibatches only (at the bench config, 16384 samples, the
        update is GPU-bound and it measured 230.3 vs 229.4 ms; config 4's 2048-sample rank minibatches: 92.3 ->
        54.6 ms per update, profiles/r04_config4_strong.jsonl).  Two graphs per minibatch -- the gradient passes,
        then clip + Adam -- with the multi-GPU gradient all-reduce issued eagerly between the two replays (no
        collective inside a captured graph).  On this path every minibatch, the eager first one included, reduces the
        whole gradient buffer with ONE flat all-reduce (`_flat_reduce`), so the replays repeat the eager step's
        arithmetic exactly on any number of ranks; the eager path's per-net buckets sum the same values, which is
        bit-identical at two ranks and can differ in the last bit from three on (ring order follows the chunking).
        tests/test_distributed_gpu.py::test_two_rank_minibatch_graphs_match_eager runs both paths on two ranks."""
        if "_mbg" not in self.__dict__:
            self._mbg = None
        if self.trace is not None or ph.on or len({len(b) for b in batches}) != 1 or self._aux_streams(2) is None:
            return False
        knob = os.environ.get("DGPPO_UPDATE_GRAPH")
        if knob is not None:
            return knob == "1"
        return len(batches[0]) * T <= self.GRAPH_MAX_SAMPLES

    def _mb_graph_key(self, rollout, det, A, Ql, Qh_det, Bm, T, L):
        ptr = lambda t: int(t.data_ptr())  # noqa: E731
        rg, dg = rollout.graph, det.graph
        fields = (rg.nodes, rg.edges, rg.receivers, rg.senders, rollout.actions, rollout.log_pis, A, Ql,
                  dg.nodes, dg.edges, dg.receivers, dg.senders, det.rnn_states, Qh_det)
        return (Bm, T, L) + tuple(ptr(f) for f in fields) + tuple(tuple(f.stride()) for f in fields)

    def _mb_capture(self, gkey, envs, args):
        """Record the minibatch step into two hipGraphs whose env-id input is a static buffer: (1) gathers and the
        three nets' passes on their streams, (2) clip + finite check + Adam; replays copy each minibatch's ids into
        the buffer, replay (1), all-reduce the gradients eagerly when there are several ranks, replay (2)."""
        static_envs = envs.clone()
        g1, g2 = K.hold_for_graph(torch.cuda.CUDAGraph()), K.hold_for_graph(torch.cuda.CUDAGraph())
        self._capturing = True
        try:
            with torch.cuda.graph(g1):
                out = self._mb_body(static_envs, *args, _Phases(self.device), apply=False)
            with torch.cuda.graph(g2):
                self._mb_apply()
        finally:
            self._capturing = False
        self._mbg = (gkey, (g1, g2), static_envs, out)

    def _mb_replay(self, envs):
        gkey, (g1, g2), static_envs, out = self._mbg
        static_envs.copy_(envs)
        g1.replay()
        self._allreduce_grads()  # eager (RCCL / gloo) between the replays; a no-op on one rank
        g2.replay()
        return out

    def _mb_apply(self):
        """clip + finite check + Adam of the three nets: two launches for all three (dgppo_adam_multi, bit-identical
        to the per-net grad_norm + adam pairs; DGPPO_ADAM_MULTI=0 runs the pairs)."""
        names = ("Vl", "Vh", "policy")
        if ADAM_MULTI() and self.device.type == "cuda":
            K.adam_multi([(o.ps.flat, o.ps.grad, o.m, o.v, o.state, o.lr, o.max_norm)
                          for o in (self.opt[k] for k in names)])
            return
        for name in names:
            self.opt[name].step()

    def _mb_body(self, envs, rollout, det, A, Ql, Qh_det, Bm, T, L, ph, apply=True):
        """One minibatch (dgppo.py:275-289): gradients of Vl, Vh and the policy on the minibatch's envs, then
        clip + finite check + Adam per net.  Device work only (capturable)."""
        env, dev, n = self._env, self.device, self._n_agents
        S_per_env = T // L
        if self.trace is not None:
            self._mb_before = dict(p={k: o.ps.flat.clone() for k, o in self.opt.items()},
                                   m={k: o.m.clone() for k, o in self.opt.items()},
                                   v={k: o.v.clone() for k, o in self.opt.items()},
                                   s={k: o.state.clone() for k, o in self.opt.items()})
        self.grad_flat.zero_()
        # the minibatch's rows of both rollouts (x[idx] of dgppo.py:278-279): two gather launches
        rg = rollout.graph
        nodes, edges, recv, send, acts, lp_old, adv, tgt = self._gather(
            envs, rg.nodes, rg.edges, rg.receivers, rg.senders, rollout.actions, rollout.log_pis, A, Ql)
        g = self._graph_batch(nodes, edges, recv, send).prepare()
        dg = det.graph
        dnodes, dedges, drecv, dsend, hd, qhd = self._gather(
            envs, dg.nodes, dg.edges, dg.receivers, dg.senders, self._rows(det.rnn_states), Qh_det)
        gd = self._graph_batch(dnodes, dedges, drecv, dsend).prepare()
        tgt = tgt.view(Bm * S_per_env, L)
        acts, lp_old, adv = acts.view(-1, self._action_dim), lp_old.view(-1), adv.view(-1)
        pending = []

        def vl_job():  # update_Vl (informarl.py:357-385)
            v, _, cache = self.Vl.seq_fwd(g, Bm * S_per_env, L)
            dv = torch.empty_like(v)
            loss = torch.empty(1, device=dev)
            K.l2_loss(v, tgt, dv, loss)
            ph.mark("Vl_fwd")
            with K.defer_wgrad(dev, self.Vl.ps.grad, DEFER_WGRAD()):
                self.Vl.seq_bwd(cache, dv)
            self._start_reduce(self.Vl, pending)  # the bucket's all-reduce overlaps the other passes
            ph.mark("Vl_bwd")
            return loss

        def vh_job():  # update_Vh (dgppo.py:296-321) on the deterministic rollout
            vh, cache = self.Vh.fwd(gd, hd.view(Bm * T * n, -1))
            dvh = torch.empty_like(vh)
            loss = torch.empty(1, device=dev)
            K.l2_loss(vh, qhd.view(-1, env.n_cost), dvh, loss)
            ph.mark("Vh_fwd")
            with K.defer_wgrad(dev, self.Vh.ps.grad, DEFER_WGRAD()):
                self.Vh.bwd(cache, dvh)
            self._start_reduce(self.Vh, pending)
            ph.mark("Vh_bwd")
            return loss

        def pi_job():  # update_policy (informarl.py:405-457)
            lp, ent, cache = self.actor.eval_seq_fwd(g, Bm * S_per_env, L, acts, self.entropy_eps)
            dlp = torch.empty_like(lp)
            dent = torch.empty_like(ent)
            st = torch.empty(4, device=dev)
            K.ppo_loss(lp, lp_old, adv, ent, self.clip_eps, self.coef_ent, dlp, dent, st)
            ph.mark("pi_fwd")
            with K.defer_wgrad(dev, self.actor.ps.grad, DEFER_WGRAD()):
                self.actor.eval_seq_bwd(cache, dlp, dent)
            self._start_reduce(self.actor, pending)
            ph.mark("pi_bwd")
            return st

        # the three passes are independent (own parameters and gradient slices): concurrent streams
        stats, vl_loss, vh_loss = self._parallel([pi_job, vl_job, vh_job])
        if not apply:  # graph capture: the caller all-reduces and runs clip + Adam from a second graph
            return vl_loss, vh_loss, stats, tgt, lp_old
        # gradient buckets all-reduced (sum, then / world), clip + finite check + Adam per net
        self._finish_reduce(pending)
        if self.trace is not None:
            self._mb_grad = self.grad_flat.clone()
        self._mb_apply()
        ph.mark("allreduce_adam")
        return vl_loss, vh_loss, stats, tgt, lp_old

    def update(self, rollout: Rollout, step: int) -> dict:
        env, dev = self._env, self.device
        B, T = rollout.rewards.shape
        n = self._n_agents
        ph = _Phases(dev)
        ph.mark()
        # DGPPO_PHASE_EVENTS=1: live (non-synchronising) split of the update into prepass / GAE + advantages /
        # minibatches from HIP events on the current stream, reported in info["time/*_ms"]
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)] if PHASE_EVENTS() and dev.type == "cuda" else None
        if ev:
            ev[0].record()
        det_key = int(self.key.integers(0, 2 ** 62))
        assert B * T * self.world >= self.batch_size
        chunk = max(1, min(B, PREPASS_GRAPHS // T))
        info = {}
        det = None
        for _ in range(self.epoch_ppo):
            # ---- prepass (dgppo.py:203-228): Vl scan over the whole episode + final Vl; Vh on every graph of
            # the rollout and of the deterministic rollout.  Independent passes on three streams: the det
            # rollout (a latency-bound 128-step launch chain) and its Vh overlap the rollout's Vl / Vh passes.
            if det is None:
                def det_job():
                    d = self.det_rollout(B, det_key)
                    return d, self._vh_all(d, chunk)

                Vl, (det, Vh_det), Vh = self._parallel([lambda: self._vl_all(rollout, chunk), det_job,
                                                        lambda: self._vh_all(rollout, chunk)])
            else:
                Vl, Vh, Vh_det = self._vl_all(rollout, chunk), self._vh_all(rollout, chunk), self._vh_all(det, chunk)
            ph.mark("prepass")
            if ev:
                ev[1].record()
            # ---- GAE + advantages
            costs = rollout.costs.contiguous()
            l = (-rollout.rewards).contiguous()
            Qh = torch.empty((B, T, n, env.n_cost), device=dev)
            Ql = self._buf("Ql", (B, T))
            K.gae(costs, l, Vh, Vl, Qh, Ql, self.gamma, self.gae_lambda)
            Qh_det = self._buf("Qh_det", (B, T, n, env.n_cost))
            Ql_det = torch.empty_like(Ql)
            K.gae(det.costs.contiguous(), (-det.rewards).contiguous(), Vh_det, Vl, Qh_det, Ql_det, self.gamma,
                  self.gae_lambda)
            A = self._buf("A", (B, T, n))
            safe_cnt = torch.empty(B, device=dev)
            # DGPPO_DEBUG_FORCE_SAFE=1 (ablation knob, not a reference option): dt = inf and alpha = 0 make
            # the CBF derivative exactly 0, so every sample counts as safe and A = -(Al + cbf_eps * w)
            dt, alpha = (math.inf, 0.0) if FORCE_SAFE() else (env.dt, self.alpha)
            K.dgppo_advantages(Ql, Vl, Vh, A, safe_cnt, dt, alpha, self.cbf_eps, self.cbf_weight_at(step))
            ph.mark("gae_adv")
            if ev:
                ev[2].record()
            if self.trace is not None:
                self.trace.update(det=det, Vl=Vl.clone(), Vh=Vh.clone(), Vh_det=Vh_det.clone(), Ql=Ql.clone(),
                                  Qh=Qh.clone(), Qh_det=Qh_det.clone(), A=A.clone(), safe_cnt=safe_cnt.clone(),
                                  mb=[])
            # ---- minibatches (dgppo.py:155-159, 275-289)
            batches = minibatch_plan(B, T, self.world, self.batch_size, self.np_rng)
            L = self.rnn_step
            assert T % L == 0, "jnp.array(jnp.array_split(...)) in the reference needs rnn_step | T"
            env_ids = self._env_ids(batches)
            graph_ok = self._mb_graph_ok(batches, ph, T)
            self._flat_reduce = graph_ok
            for k, bi in enumerate(batches):
                envs = next(env_ids)
                args = (rollout, det, A, Ql, Qh_det, len(bi), T, L)
                if graph_ok:
                    gkey = self._mb_graph_key(*args)
                    if self._mbg is not None and self._mbg[0] == gkey:
                        out = self._mb_replay(envs)
                    else:
                        out = self._mb_body(envs, *args, ph)  # the first minibatch runs eagerly, then capture
                        self._mb_capture(gkey, envs, args)
                else:
                    out = self._mb_body(envs, *args, ph)
                vl_loss, vh_loss, stats, tgt, lp_old = out
                if self.trace is not None:
                    self.trace["mb"].append(dict(
                        envs=bi.copy(), grad=self._mb_grad, vl_loss=vl_loss.clone(), vh_loss=vh_loss.clone(),
                        stats=stats.clone(), before=self._mb_before["p"], m_before=self._mb_before["m"],
                        v_before=self._mb_before["v"], state_before=self._mb_before["s"]))
            self._flat_reduce = False
            info = {"Vl/loss": vl_loss, "Vl/max_target": tgt.max(), "Vl/min_target": tgt.min(),
                    "Vh/loss_Vh": vh_loss, "policy/stats": stats, "policy/log_pi_min": lp_old.min()}
            safe = safe_cnt.sum()
            if self._reduce:
                dist.all_reduce(safe)
            info["eval/safe_data"] = safe / (B * self.world * T * n)
            # learning diagnostics (not reference metrics): per cost column, the mean Vh over the rollout's
            # graphs, the det rollout's Vh / Qh_det targets and its costs -- one device vector, one copy
            info["diag/vec"] = torch.cat([Vh[:, :T].mean((0, 1, 2)), Vh_det[:, :T].mean((0, 1, 2)),
                                          Qh_det.mean((0, 1, 2)), det.costs.mean((0, 1, 2))])
        ph.report()
        if ev:
            ev[3].record()
            ev[3].synchronize()
            for name, a, b in (("prepass", 0, 1), ("gae_adv", 1, 2), ("minibatches", 2, 3)):
                info[f"time/{name}_ms"] = ev[a].elapsed_time(ev[b])
        return self._finish_info(info)

    def _finish_info(self, info) -> dict:
        out = {}
        st = info.pop("policy/stats", None)
        dv = info.pop("diag/vec", None)
        if dv is not None:
            nh = self._env.n_cost
            d = dv.cpu().numpy().reshape(4, nh)
            for i, tag in enumerate(("Vh/mean", "Vh/det_mean", "Vh/det_target_mean", "det/cost_mean")):
                for j in range(nh):
                    out[f"{tag}_h{j}"] = float(d[i, j])
        for k, v in info.items():
            out[k] = float(v.reshape(-1)[0].item()) if torch.is_tensor(v) else v
        if st is not None:
            s = st.cpu().numpy()
            out["policy/loss"] = float(s[0] - self.coef_ent * s[1])
            out["policy/entropy"], out["policy/clip_frac"], out["policy/total_variation_dist"] = \
                float(s[1]), float(s[2]), float(0.5 * s[3])
        for name, tag in (("Vl", "Vl/grad_norm"), ("Vh", "Vh/grad_Vh_norm"), ("policy", "policy/grad_norm")):
            stv = self.opt[name].state.cpu().numpy()
            out[tag] = float(stv[0])
            out[{"Vl": "Vl/has_nan", "Vh": "Vh/grad_Vh_has_nan", "policy": "policy/has_nan"}[name]] = float(stv[1] > 0)
        return out

    # ---- checkpoints ---------------------------------------------------------------------------
    def save(self, save_dir: str, step: int):
        """models/<step>/{actor,Vl,Vh}.pt: params AND Adam state (the reference keeps params only)."""
        d = os.path.join(save_dir, str(step))
        os.makedirs(d, exist_ok=True)
        for name, net, opt in (("actor", self.actor, self.opt["policy"]), ("Vl", self.Vl, self.opt["Vl"]),
                               ("Vh", self.Vh, self.opt["Vh"])):
            torch.save({"params": net.ps.flat.cpu(), "m": opt.m.cpu(), "v": opt.v.cpu(), "state": opt.state.cpu(),
                        "layout": [(n, s) for n, s, _ in net.ps.entries]}, os.path.join(d, f"{name}.pt"))

    def load(self, load_dir: str, step: int):
        """models/<step>/{actor,Vl,Vh}.pt of this package, or reference-layout {actor,Vl,Vh}.npz flax
        trees (utils/flax_ckpt.py; params only, Adam state kept)."""
        d = os.path.join(load_dir, str(step))
        if not os.path.exists(os.path.join(d, "actor.pt")) and os.path.exists(os.path.join(d, "actor.npz")):
            from ..utils.flax_ckpt import load_reference_npz

            load_reference_npz(self, d)
            return
        for name, net, opt in (("actor", self.actor, self.opt["policy"]), ("Vl", self.Vl, self.opt["Vl"]),
                               ("Vh", self.Vh, self.opt["Vh"])):
            ck = torch.load(os.path.join(d, f"{name}.pt"), weights_only=True)
            net.ps.flat.copy_(ck["params"])
            opt.m.copy_(ck["m"]), opt.v.copy_(ck["v"]), opt.state.copy_(ck["state"])

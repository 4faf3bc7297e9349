"""PyTorch-ROCm custom ops over libdgppo_hip.so: `torch.ops.dgppo.*`.

The hot-path kernels are registered with `torch.library` so the torch dispatcher, FakeTensor /
meta tracing (torch.compile, export) and CUDA-graph capture all see them as ordinary ops.  Each op
is a thin shim over the C-ABI entry point declared in include/dgppo_hip.h (the same function a
cgo / JNI / ctypes binding would call); outputs are caller-allocated and written
in place (`mutates_args`), launches go on torch's current stream, and there is no CPU kernel: a
non-CUDA tensor raises NativeLibraryError (`_lib.require_gpu`).

  dgppo::env_reset      dgppo_env_reset      vmap(env.reset)      lidar_env/base.py:89-124, mpe/base.py:81-127
  dgppo::env_step       dgppo_env_step       vmap(env.step)       lidar_env/base.py:151-174, mpe/base.py:137-158
  dgppo::env_reset_states dgppo_env_reset_states  the sampling half of env_reset (no graph)
  dgppo::env_rollout    dgppo_env_rollout    lax.scan of env.step over T given actions, trainer/utils.py:45-55
  dgppo::gnn_attn_fwd   dgppo_gnn_attn_fwd   GraphTransformer attention core, gnn.py:83-117
  dgppo::gnn_attn_bwd   dgppo_gnn_attn_bwd   its gradient (the jax.grad of update_Vl / update_policy)
  dgppo::gae            dgppo_gae            compute_dec_ocp_gae, algo/utils.py:11-79
  dgppo::grad_norm      dgppo_grad_norm      compute_norm + has_any_nan_or_inf, trainer/utils.py:105-118
  dgppo::adam           dgppo_adam           clip + optax.apply_if_finite(optax.adam), informarl.py:131-137
  dgppo::gather_env_steps dgppo_gather_env_steps  tree_map(lambda x: x[idx], rollout), dgppo.py:275-289

An env's static configuration (dgppo_env_cfg: engine, sizes, radii, limits) is not a tensor; it is
registered once per env instance and the ops take its integer handle.
"""
from __future__ import annotations

import ctypes
import itertools
import weakref
from typing import List, Optional

import torch
from torch import Tensor

from . import _lib

_CFGS: dict = {}
_NEXT_HANDLE = itertools.count(1)


def register_env_cfg(cfg: _lib.EnvCfg, owner=None) -> int:
    """Keep `cfg` alive and return the handle the env ops take (handles are never reused).  With an
    `owner` the entry is released when the owner is garbage-collected, so per-test / per-config envs
    do not accumulate for the life of the process."""
    h = next(_NEXT_HANDLE)
    _CFGS[h] = cfg
    if owner is not None:
        weakref.finalize(owner, _CFGS.pop, h, None)
    return h


def env_cfg(handle: int) -> _lib.EnvCfg:
    try:
        return _CFGS[int(handle)]
    except KeyError:
        raise ValueError(f"unknown env cfg handle {handle}") from None


def _stride(t: Tensor, inner: int) -> int:
    """Per-env element stride of t, requiring the trailing `inner` dims to be contiguous."""
    tail = 1
    for d in range(t.dim() - 1, t.dim() - 1 - inner, -1):
        if t.stride(d) != tail:
            raise ValueError("trailing dims must be contiguous")
        tail *= t.shape[d]
    return t.stride(t.dim() - 1 - inner) if t.dim() > inner else tail


def _p(t: Optional[Tensor]) -> int:
    return 0 if t is None else int(t.data_ptr())


def _stream(t: Tensor) -> int:
    return _lib.stream_handle(t.device)


# ---- env -------------------------------------------------------------------------------------------
@torch.library.custom_op("dgppo::env_step", mutates_args=("nodes", "edges", "out_states", "receivers", "senders",
                                                           "reward", "cost"))
def env_step(cfg: int, states: Tensor, obstacles: Optional[Tensor], action: Tensor, ray_dirs: Tensor, nodes: Tensor,
             edges: Tensor, out_states: Tensor, receivers: Tensor, senders: Tensor, reward: Tensor,
             cost: Tensor) -> None:
    """One fused env step for B envs: states (B, N, sd) [+ obstacles (B, O, 16)] and actions (B, n, A)
    -> next graph rows, reward (B,), cost (B, n, n_cost).  Per-env strides are free (views into a
    time-major rollout buffer); the trailing dims must be contiguous."""
    _lib.require_gpu(states.device, "dgppo::env_step")
    io = _lib.EnvStepIO()
    io.states, io.states_stride = _p(states), _stride(states, 2)
    io.obstacles = _p(obstacles)
    io.obstacles_stride = obstacles.stride(-3) if obstacles is not None else 0
    io.action, io.action_stride = _p(action), _stride(action, 2)
    io.ray_dirs = _p(ray_dirs)
    io.nodes, io.nodes_stride = _p(nodes), _stride(nodes, 2)
    io.edges, io.edges_stride = _p(edges), _stride(edges, 2)
    io.out_states, io.out_states_stride = _p(out_states), _stride(out_states, 2)
    io.receivers, io.senders = _p(receivers), _p(senders)
    io.edge_index_stride = _stride(receivers, 1)
    io.reward, io.reward_stride = _p(reward), (reward.stride(0) if reward.dim() > 0 else 1)
    io.cost, io.cost_stride = _p(cost), _stride(cost, 2)
    io.n_env = int(states.shape[0])
    _lib.check(_lib.load().dgppo_env_step(ctypes.byref(env_cfg(cfg)), ctypes.byref(io), _stream(states)),
               "dgppo_env_step")


@env_step.register_fake
def _env_step_fake(cfg, states, obstacles, action, ray_dirs, nodes, edges, out_states, receivers, senders, reward,
                   cost) -> None:
    return None


@torch.library.custom_op("dgppo::env_reset", mutates_args=("obstacles", "nodes", "edges", "out_states", "receivers",
                                                            "senders"))
def env_reset(cfg: int, key: Optional[Tensor], seed: int, env_offset: int, n_env: int, obstacles: Optional[Tensor],
              ray_dirs: Tensor, nodes: Tensor, edges: Tensor, out_states: Tensor, receivers: Tensor,
              senders: Tensor) -> None:
    """Reset n_env envs (env b draws from Philox keyed (seed or *key, env_offset + b)) and write the
    initial graph.  `key`: optional 1-element int64 device tensor read at run time (hipGraph replays)."""
    _lib.require_gpu(nodes.device, "dgppo::env_reset")
    io = _reset_io(key, seed, env_offset, n_env, obstacles, ray_dirs, nodes, edges, out_states, receivers, senders)
    _lib.check(_lib.load().dgppo_env_reset(ctypes.byref(env_cfg(cfg)), ctypes.byref(io), _stream(nodes)),
               "dgppo_env_reset")


@env_reset.register_fake
def _env_reset_fake(cfg, key, seed, env_offset, n_env, obstacles, ray_dirs, nodes, edges, out_states, receivers,
                    senders) -> None:
    return None


def _reset_io(key, seed, env_offset, n_env, obstacles, ray_dirs, nodes, edges, out_states, receivers, senders):
    io = _lib.EnvResetIO()
    if key is not None:
        if key.device != out_states.device or key.numel() != 1 or key.dtype not in (torch.int64, torch.uint64):
            raise ValueError("tensor key must be a 1-element int64 tensor on the env's device")
        io.seed, io.seed_ptr = 0, key.data_ptr()
    else:
        io.seed, io.seed_ptr = int(seed) & 0xFFFFFFFFFFFFFFFF, None
    io.env_offset = int(env_offset)
    io.obstacles = _p(obstacles)
    io.obstacles_stride = obstacles.stride(0) if obstacles is not None else 0
    io.ray_dirs = _p(ray_dirs)
    io.nodes, io.nodes_stride = _p(nodes), _stride(nodes, 2)
    io.edges, io.edges_stride = _p(edges), _stride(edges, 2)
    io.out_states, io.out_states_stride = _p(out_states), _stride(out_states, 2)
    io.receivers, io.senders = _p(receivers), _p(senders)
    io.edge_index_stride = _stride(receivers, 1)
    io.n_env = int(n_env)
    return io


@torch.library.custom_op("dgppo::env_reset_states", mutates_args=("obstacles", "nodes", "edges", "out_states",
                                                                   "receivers", "senders"))
def env_reset_states(cfg: int, key: Optional[Tensor], seed: int, env_offset: int, n_env: int,
                     obstacles: Optional[Tensor], ray_dirs: Tensor, nodes: Tensor, edges: Tensor, out_states: Tensor,
                     receivers: Tensor, senders: Tensor) -> None:
    """env_reset's sampling half: obstacle records and agent / goal state rows (configs without the
    persistent rollout kernel: the full reset).  Pair with env_rollout(rebuild_first=True)."""
    _lib.require_gpu(out_states.device, "dgppo::env_reset_states")
    io = _reset_io(key, seed, env_offset, n_env, obstacles, ray_dirs, nodes, edges, out_states, receivers, senders)
    _lib.check(_lib.load().dgppo_env_reset_states(ctypes.byref(env_cfg(cfg)), ctypes.byref(io), _stream(out_states)),
               "dgppo_env_reset_states")


@env_reset_states.register_fake
def _env_reset_states_fake(cfg, key, seed, env_offset, n_env, obstacles, ray_dirs, nodes, edges, out_states,
                           receivers, senders) -> None:
    return None


@torch.library.custom_op("dgppo::env_rollout", mutates_args=("nodes", "edges", "states", "receivers", "senders",
                                                              "reward", "cost"))
def env_rollout(cfg: int, rebuild_first: bool, obstacles: Optional[Tensor], actions: Tensor, ray_dirs: Tensor,
                nodes: Tensor, edges: Tensor, states: Tensor, receivers: Tensor, senders: Tensor, reward: Tensor,
                cost: Tensor) -> None:
    """T env steps with given actions (T, B, n, A) through time-major graph buffers (T+1, B, ...):
    step t reads graph t and writes graph t+1, reward[t] (T, B), cost[t] (T, B, n, n_cost).
    rebuild_first: graph 0's rows are first built from its agent / goal states (env_reset_states)."""
    _lib.require_gpu(states.device, "dgppo::env_rollout")
    T = int(actions.shape[0])
    if states.shape[0] != T + 1 or reward.shape[0] != T or cost.shape[0] != T:
        raise ValueError("env_rollout: graph buffers must hold T+1 graphs, actions / reward / cost T steps")
    r = _lib.EnvRolloutIO()
    io = r.step
    io.states, io.states_stride = _p(states), _stride(states[0], 2)
    io.obstacles = _p(obstacles)
    io.obstacles_stride = obstacles.stride(-3) if obstacles is not None else 0
    io.action, io.action_stride = _p(actions), _stride(actions[0], 2)
    io.ray_dirs = _p(ray_dirs)
    io.nodes, io.nodes_stride = _p(nodes), _stride(nodes[0], 2)
    io.edges, io.edges_stride = _p(edges), _stride(edges[0], 2)
    io.out_states, io.out_states_stride = _p(states), _stride(states[0], 2)
    io.receivers, io.senders = _p(receivers), _p(senders)
    io.edge_index_stride = _stride(receivers[0], 1)
    io.reward, io.reward_stride = _p(reward), reward.stride(1)
    io.cost, io.cost_stride = _p(cost), _stride(cost[0], 2)
    io.n_env = int(states.shape[1])
    r.T, r.rebuild_first = T, int(bool(rebuild_first))
    r.t_states, r.t_nodes, r.t_edges = states.stride(0), nodes.stride(0), edges.stride(0)
    if receivers.stride(0) != senders.stride(0):
        raise ValueError("env_rollout: receivers and senders need the same time stride")
    r.t_index, r.t_action, r.t_reward, r.t_cost = receivers.stride(0), actions.stride(0), reward.stride(0), cost.stride(0)
    _lib.check(_lib.load().dgppo_env_rollout(ctypes.byref(env_cfg(cfg)), ctypes.byref(r), _stream(states)),
               "dgppo_env_rollout")


@env_rollout.register_fake
def _env_rollout_fake(cfg, rebuild_first, obstacles, actions, ray_dirs, nodes, edges, states, receivers, senders,
                      reward, cost) -> None:
    return None


# ---- GraphTransformer attention core -------------------------------------------------------------------
def _attn_struct(dims, cand, receivers, senders, sidx, x, x_gstride, ef, ef_gstride, q, qt, bk, scale, xa, xa_gstride,
                 pre_W, pre_b, beta=None, beta_ld=0, qt_ld=0) -> _lib.GnnAttnArgs:
    a = _lib.GnnAttnArgs()
    a.G, a.N, a.E, a.n_agents, a.D, a.F, a.H, a.C, a.D0 = (int(v) for v in dims)
    a.cand, a.receivers, a.senders, a.sidx = _p(cand), _p(receivers), _p(senders), _p(sidx)
    a.x, a.x_gstride = _p(x), int(x_gstride)
    a.ef, a.ef_gstride = _p(ef), int(ef_gstride)
    a.q, a.qt, a.bk = _p(q), _p(qt), _p(bk)
    a.scale = float(scale)
    a.xa, a.xa_gstride = _p(xa), int(xa_gstride)
    a.pre_W, a.pre_b = _p(pre_W), _p(pre_b)
    a.beta, a.beta_ld, a.qt_ld = _p(beta), int(beta_ld), int(qt_ld)
    return a


@torch.library.custom_op("dgppo::gnn_attn_fwd", mutates_args=("attn", "xcat"))
def gnn_attn_fwd(dims: List[int], cand: Tensor, receivers: Tensor, senders: Tensor, sidx: Tensor, x: Tensor,
                 x_gstride: int, ef: Tensor, ef_gstride: int, q: Optional[Tensor], qt: Tensor, bk: Tensor,
                 scale: float, xa: Optional[Tensor], xa_gstride: int, pre_W: Optional[Tensor],
                 pre_b: Optional[Tensor], attn: Tensor, xcat: Tensor, beta: Optional[Tensor] = None,
                 beta_ld: int = 0, qt_ld: int = 0) -> None:
    """Per-receiving-agent attention of one GraphTransformer layer (dims = [G, N, E, n, D, F, H, C, D0]):
    attn (G*n, H, C) = segment softmax of (q . k)/sqrt(F) over each agent's candidate edges, xcat
    (G*n, H*(D+5)) = the attention-weighted [sender rows | edge rows | 1] per head (nn/layers.py).
    Q-free form: q None and beta (G*n, H) = q_h . bk_h given (row stride beta_ld); qt_ld = qt's row stride."""
    _lib.require_gpu(qt.device, "dgppo::gnn_attn_fwd")
    a = _attn_struct(dims, cand, receivers, senders, sidx, x, x_gstride, ef, ef_gstride, q, qt, bk, scale, xa,
                     xa_gstride, pre_W, pre_b, beta, beta_ld, qt_ld)
    a.attn, a.xcat = _p(attn), _p(xcat)
    _lib.check(_lib.load().dgppo_gnn_attn_fwd(ctypes.byref(a), _stream(qt)), "dgppo_gnn_attn_fwd")


@gnn_attn_fwd.register_fake
def _gnn_attn_fwd_fake(dims, cand, receivers, senders, sidx, x, x_gstride, ef, ef_gstride, q, qt, bk, scale, xa,
                       xa_gstride, pre_W, pre_b, attn, xcat, beta=None, beta_ld=0, qt_ld=0) -> None:
    return None


@torch.library.custom_op("dgppo::gnn_attn_bwd", mutates_args=("dqt", "dq", "dbeta", "dxa", "dpre_part", "dx"))
def gnn_attn_bwd(dims: List[int], cand: Tensor, receivers: Tensor, senders: Tensor, sidx: Tensor, x: Tensor,
                 x_gstride: int, ef: Tensor, ef_gstride: int, q: Optional[Tensor], qt: Tensor, bk: Tensor,
                 scale: float, xa: Optional[Tensor], xa_gstride: int, pre_W: Optional[Tensor],
                 pre_b: Optional[Tensor], attn: Tensor, dxcat: Tensor, da_add: Optional[Tensor], dqt: Tensor,
                 dq: Optional[Tensor], dbeta: Tensor, dxa: Optional[Tensor], dxa_gstride: int,
                 dpre_part: Optional[Tensor], beta: Optional[Tensor] = None, beta_ld: int = 0, qt_ld: int = 0,
                 dqt_ld: int = 0, dbeta_ld: int = 0, dx: Optional[Tensor] = None, dx_gstride: int = 0) -> None:
    """Backward of gnn_attn_fwd given dL/dxcat (+ da_add, extra dL/dattn of edge columns past 4): dqt, dq,
    dbeta (dL/d(q . bk)); in agent mode dxa (accumulated, agent senders) and the partial Dense_4
    gradients of the recomputed never-receiving senders (dpre_part, one row per workgroup); otherwise,
    if dx is given, the sender gradient of every node row of x (accumulated, graph stride dx_gstride).
    Q-free form: dq None (not written), dqt / dbeta row strides dqt_ld / dbeta_ld (e.g. one [dqt | dbeta]
    buffer)."""
    _lib.require_gpu(qt.device, "dgppo::gnn_attn_bwd")
    a = _attn_struct(dims, cand, receivers, senders, sidx, x, x_gstride, ef, ef_gstride, q, qt, bk, scale, xa,
                     xa_gstride, pre_W, pre_b, beta, beta_ld, qt_ld)
    a.dqt_ld, a.dbeta_ld = int(dqt_ld), int(dbeta_ld)
    a.attn, a.dxcat, a.da_add = _p(attn), _p(dxcat), _p(da_add)
    a.dqt, a.dq, a.dbeta = _p(dqt), _p(dq), _p(dbeta)
    a.dxa, a.dxa_gstride, a.dpre_part = _p(dxa), int(dxa_gstride), _p(dpre_part)
    a.dx, a.dx_gstride = _p(dx), int(dx_gstride)
    _lib.check(_lib.load().dgppo_gnn_attn_bwd(ctypes.byref(a), _stream(qt)), "dgppo_gnn_attn_bwd")


@gnn_attn_bwd.register_fake
def _gnn_attn_bwd_fake(dims, cand, receivers, senders, sidx, x, x_gstride, ef, ef_gstride, q, qt, bk, scale, xa,
                       xa_gstride, pre_W, pre_b, attn, dxcat, da_add, dqt, dq, dbeta, dxa, dxa_gstride, dpre_part,
                       beta=None, beta_ld=0, qt_ld=0, dqt_ld=0, dbeta_ld=0, dx=None, dx_gstride=0) -> None:
    return None


def gnn_attn_partial_blocks(dims, cand, receivers, senders, sidx, x, x_gstride, ef, ef_gstride, q, qt, bk, scale, xa,
                            xa_gstride, pre_W, pre_b, beta=None, beta_ld=0, qt_ld=0) -> int:
    """Rows of the dpre_part workspace gnn_attn_bwd writes for these arguments (host query)."""
    a = _attn_struct(dims, cand, receivers, senders, sidx, x, x_gstride, ef, ef_gstride, q, qt, bk, scale, xa,
                     xa_gstride, pre_W, pre_b, beta, beta_ld, qt_ld)
    return int(_lib.load().dgppo_gnn_attn_partial_blocks(ctypes.byref(a)))


# ---- one GraphTransformer layer forward as one kernel (ABI 11) -------------------------------------------
TAIL_FIELDS = ("W0", "b0", "ln0_s", "ln0_b", "W1", "b1", "ln1_s", "ln1_b", "Wi", "bi", "Wh", "bhn", "Wo", "bo")


def _layer_struct(dims, cand, receivers, senders, sidx, x, x_gstride, ef, ef_gstride, scale, xa, xa_gstride, pre_W,
                  pre_b, QBW, Wcat, Wu, bu, Y, qb=None, attn=None, xcat=None, zmean=None, tail_w=(), tail_h=None,
                  tail_out=None) -> _lib.GnnLayerArgs:
    la = _lib.GnnLayerArgs()
    la.a = _attn_struct(dims, cand, receivers, senders, sidx, x, x_gstride, ef, ef_gstride, None, None, None, scale, xa,
                        xa_gstride, pre_W, pre_b)
    la.a.attn, la.a.xcat = _p(attn), _p(xcat)
    la.QBW, la.qb, la.Wcat, la.Wu, la.bu, la.Y = _p(QBW), _p(qb), _p(Wcat), _p(Wu), _p(bu), _p(Y)
    la.zmean = _p(zmean)
    if tail_out is not None:
        for name, t in zip(TAIL_FIELDS, tail_w):
            setattr(la.tail, name, _p(t))
        la.tail.h_in, la.tail.out = _p(tail_h), _p(tail_out)
        la.tail.n_out, la.tail.on = int(tail_out.shape[-1]), 1
    return la


def gnn_layer_supported(**kw) -> bool:
    """Whether dgppo_gnn_layer_fwd covers this layer call (host query; same keyword arguments as gnn_layer_fwd)."""
    return bool(_lib.load().dgppo_gnn_layer_supported(ctypes.byref(_layer_struct(**kw))))


@torch.library.custom_op("dgppo::gnn_layer_fwd", mutates_args=("Y", "qb", "attn", "xcat", "zmean", "tail_out"))
def gnn_layer_fwd(dims: List[int], cand: Tensor, receivers: Tensor, senders: Tensor, sidx: Tensor, x: Tensor,
                  x_gstride: int, ef: Tensor, ef_gstride: int, scale: float, xa: Optional[Tensor], xa_gstride: int,
                  pre_W: Optional[Tensor], pre_b: Optional[Tensor], QBW: Tensor, Wcat: Tensor, Wu: Tensor, bu: Tensor,
                  Y: Optional[Tensor], qb: Optional[Tensor], attn: Optional[Tensor], xcat: Optional[Tensor],
                  zmean: Optional[Tensor], tail_w: List[Tensor], tail_h: Optional[Tensor],
                  tail_out: Optional[Tensor]) -> None:
    """One GraphTransformer layer forward (dims as gnn_attn_fwd): Y (G*n, F) = relu(xcat Wcat / H + x_i Wu + bu) with
    the attention of gnn_attn_fwd in between and [qt | beta] = [x_i 1] QBW, all in one kernel; qb, attn and xcat are
    optional outputs for the backward (nn/layers.py GraphTransformer.fwd).  Forward-only epilogues: zmean (G, F) the
    per-graph agent mean of Y; tail_out (G*n, n_out) the value head after the layer (MLP -> GRU(tail_h) -> Dense,
    weights tail_w in TAIL_FIELDS order)."""
    dev = (Y if Y is not None else zmean if zmean is not None else tail_out).device
    _lib.require_gpu(dev, "dgppo::gnn_layer_fwd")
    la = _layer_struct(dims, cand, receivers, senders, sidx, x, x_gstride, ef, ef_gstride, scale, xa, xa_gstride, pre_W,
                       pre_b, QBW, Wcat, Wu, bu, Y, qb, attn, xcat, zmean, tail_w, tail_h, tail_out)
    _lib.check(_lib.load().dgppo_gnn_layer_fwd(ctypes.byref(la), _lib.stream_handle(dev)), "dgppo_gnn_layer_fwd")


@gnn_layer_fwd.register_fake
def _gnn_layer_fwd_fake(dims, cand, receivers, senders, sidx, x, x_gstride, ef, ef_gstride, scale, xa, xa_gstride,
                        pre_W, pre_b, QBW, Wcat, Wu, bu, Y, qb, attn, xcat, zmean, tail_w, tail_h, tail_out) -> None:
    return None


# ---- GAE, clip + Adam ------------------------------------------------------------------------------------
@torch.library.custom_op("dgppo::gae", mutates_args=("Qh", "Ql"))
def gae(hs: Tensor, l: Tensor, Vh: Tensor, Vl: Tensor, Qh: Tensor, Ql: Tensor, gamma: float, lam: float) -> None:
    """Dec-OCP GAE per env: hs (B, T, n, nh) costs, l (B, T) losses, Vh (B, T+1, n, nh), Vl (B, T+1)
    -> Qh (B, T, n, nh), Ql (B, T) (the reference's O(T^2) row scan, literally)."""
    _lib.require_gpu(hs.device, "dgppo::gae")
    for t in (hs, l, Vh, Vl, Qh, Ql):
        if not t.is_contiguous():
            raise ValueError("dgppo::gae needs contiguous tensors")
    B, T, n, nh = hs.shape
    a = _lib.GaeArgs()
    a.B, a.T, a.n_agents, a.n_h = int(B), int(T), int(n), int(nh)
    a.hs, a.l, a.Vh, a.Vl, a.Qh, a.Ql = _p(hs), _p(l), _p(Vh), _p(Vl), _p(Qh), _p(Ql)
    a.gamma = float(gamma)
    setattr(a, "lambda", float(lam))
    _lib.check(_lib.load().dgppo_gae(ctypes.byref(a), _stream(hs)), "dgppo_gae")


@gae.register_fake
def _gae_fake(hs, l, Vh, Vl, Qh, Ql, gamma, lam) -> None:
    return None


@torch.library.custom_op("dgppo::grad_norm", mutates_args=("state",))
def grad_norm(grad: Tensor, state: Tensor) -> None:
    """state[0] = global L2 norm of grad, state[1] = number of non-finite entries (state[2]: Adam count)."""
    _lib.require_gpu(grad.device, "dgppo::grad_norm")
    lib = _lib.load()
    from .nn.kernels import workspace

    ws = workspace(lib.dgppo_loss_workspace_floats(), grad.device, "norm")
    _lib.check(lib.dgppo_grad_norm(_p(grad), int(grad.numel()), _p(state), _p(ws), _stream(grad)), "dgppo_grad_norm")


@grad_norm.register_fake
def _grad_norm_fake(grad, state) -> None:
    return None


@torch.library.custom_op("dgppo::adam", mutates_args=("param", "m", "v", "state"))
def adam(param: Tensor, grad: Tensor, m: Tensor, v: Tensor, state: Tensor, lr: float, b1: float, b2: float,
         eps: float, max_norm: float) -> None:
    """g <- g * max_norm / max(max_norm, |g|) and one optax adam step, skipped entirely (apply_if_finite)
    when state[1] (non-finite count from dgppo::grad_norm) is non-zero; state[2] counts applied steps."""
    _lib.require_gpu(param.device, "dgppo::adam")
    _lib.check(_lib.load().dgppo_adam(_p(param), _p(grad), _p(m), _p(v), int(param.numel()), _p(state), float(lr),
                                      float(b1), float(b2), float(eps), float(max_norm), _stream(param)), "dgppo_adam")


@adam.register_fake
def _adam_fake(param, grad, m, v, state, lr, b1, b2, eps, max_norm) -> None:
    return None


# ---- minibatch assembly ---------------------------------------------------------------------------------
@torch.library.custom_op("dgppo::gather_env_steps", mutates_args=("dst",))
def gather_env_steps(src: List[Tensor], dst: List[Tensor], envs: Tensor) -> None:
    """dst[i][e, t] = src[i][envs[e], t] for (B, T, ...) rollout fields (any strides on B and T, e.g. views
    of time-major buffers; contiguous trailing dims; 4-byte dtypes) into contiguous (Bm, T, ...) outputs:
    the reference's `jtu.tree_map(lambda x: x[idx], rollout)` as one launch for up to 8 fields."""
    if not src or len(src) != len(dst) or len(src) > 8:
        raise ValueError("gather_env_steps: 1..8 (src, dst) pairs")
    _lib.require_gpu(envs.device, "dgppo::gather_env_steps")
    if envs.dtype != torch.int64 or envs.dim() != 1:
        raise ValueError("envs must be a 1-d int64 tensor")
    T = int(src[0].shape[1])
    fields = (_lib.GatherField * len(src))()
    for f, a, b in zip(fields, src, dst):
        if a.element_size() != 4 or b.element_size() != 4 or a.dim() < 2 or a.shape[1] != T:
            raise ValueError("gather_env_steps: (B, T, ...) fields of 4-byte elements")
        if tuple(b.shape) != (envs.shape[0],) + tuple(a.shape[1:]) or not b.is_contiguous():
            raise ValueError("gather_env_steps: dst must be contiguous (len(envs), T, ...)")
        inner = 1
        for d in range(a.dim() - 1, 1, -1):
            if a.shape[d] != 1 and a.stride(d) != inner:
                raise ValueError("gather_env_steps: trailing dims must be contiguous")
            inner *= a.shape[d]
        f.src, f.dst, f.row_elems = _p(a), _p(b), inner
        f.src_tstride, f.src_estride = a.stride(1), a.stride(0)
    _lib.check(_lib.load().dgppo_gather_env_steps(fields, len(src), _p(envs), int(envs.shape[0]), T, _stream(envs)),
               "dgppo_gather_env_steps")


@gather_env_steps.register_fake
def _gather_env_steps_fake(src, dst, envs) -> None:
    return None

"""The three DGPPO networks with explicit forward/backward:

  ActorNet  PPOPolicy / TanhNormal / PolicyNet (dgppo/algo/module/policy.py:20-212):
            GraphTransformerGNN(2 layers, 32 -> 64, 3 heads) -> MLP(64,64)+LN -> GRUCell(64) ->
            ScaleHid Dense(64, init x0.01, no activation) -> mean Dense(2), std Dense(2) ->
            std = softplus(x + log(e^0.5 - 1)) + 1e-5 -> Independent(TanhTransformed(Normal)).
  VlNet     ValueNet(decompose=False) = RStateFn (dgppo/algo/module/value.py:15-44): GNN(2 layers)
            -> mean over agents -> MLP -> GRUCell -> Dense(1).
  VhNet     DGPPO's ValueNet(n_out=n_cost, gnn_layers=1, decompose=True, use_global_info=False) =
            DecRStateFn (value.py:47-79, dgppo.py:83-95): GNN(1 layer) -> MLP -> GRUCell fed the
            ACTOR's stored carry -> Dense(n_cost).

Rows are always ordered (graph, agent).  Sequences (the 16-step truncated-BPTT chunks of
informarl.py:365-367 / 409-413) are (sequence s, step t) graph-major, carries start at zero.
"""
from __future__ import annotations

import ctypes
import math
import os

import numpy as np
import torch

from ... import _lib
from ...nn import kernels as K
from ...nn.layers import FUSE_LN, GNN, Dense, GraphBatch, MLPHead, ParamSpace, RNNStack

# the whole forward-only get_Vh in the GNN layer's kernel (its value-head tail): measured slower than the layer kernel +
# the unfused head GEMMs (418 vs ~334 us per 131k agent rows: every 16-row workgroup reloads the head / GRU weights
# from L2), so off unless DGPPO_VH_TAIL=1
VH_TAIL = os.environ.get("DGPPO_VH_TAIL", "0") == "1"
STD_DEV_INIT_INV = math.log(math.exp(0.5) - 1.0)  # TanhNormal.std_dev_init_inv (policy.py:54-59)
STD_DEV_MIN = 1e-5


class _Net:
    modules: list

    def init_host(self, seed: int):
        rng = np.random.default_rng(seed)
        for m in self.modules:
            m.init_host(rng)

    @property
    def n_params(self):
        return self.ps.size

    @property
    def carry_width(self) -> int:
        """floats per agent carry row: (rnn_layers, carries, 64) flattened (64 for the 1-layer GRU default)."""
        return self.gru.W


class ActorNet(_Net):
    def __init__(self, node_dim: int, n_agents: int, device, seed: int = 0, gnn_layers: int = 2, action_dim: int = 2,
                 edge_dim: int = 4, rnn: str = "gru", rnn_layers: int = 1):
        self.n, self.A = n_agents, action_dim
        self.node_dim, self.edge_dim = node_dim, edge_dim
        ps = self.ps = ParamSpace()
        self.gnn = GNN(ps, "gnn", node_dim, gnn_layers, edge_dim=edge_dim)
        self.head = MLPHead(ps, "head")
        self.gru = RNNStack(ps, "gru", rnn, rnn_layers)  # RNN(GRUCell | LSTMCell, layers) or none
        self.scale_hid = Dense(ps, "ScaleHid", 64, 64, scale=0.01)
        self.mean = Dense(ps, "OutputDenseMean", 64, action_dim)
        self.std = Dense(ps, "OutputDenseStdTrans", 64, action_dim)
        self.modules = [self.gnn, self.head, self.gru, self.scale_hid, self.mean, self.std]
        ps.build(device)
        self.init_host(seed)
        self.device = torch.device(device)

    # flax-layout import / export (checkpoint interop and oracle tests)
    def flax(self):
        return {"gnn": self.gnn.flax(), "head": self.head.flax(), "gru": self.gru.flax(),
                "ScaleHid": self.scale_hid.flax(), "OutputDenseMean": self.mean.flax(),
                "OutputDenseStdTrans": self.std.flax()}

    def load_flax(self, d):
        self.gnn.load_flax(d["gnn"]), self.head.load_flax(d["head"]), self.gru.load_flax(d["gru"])
        self.scale_hid.load_flax(d["ScaleHid"]), self.mean.load_flax(d["OutputDenseMean"])
        self.std.load_flax(d["OutputDenseStdTrans"])

    def _trunk(self, g: GraphBatch, keep=True):
        z, gc = self.gnn.fwd(g, keep=keep)
        y, hc = self.head.fwd(z)
        return y, (gc, hc)

    def _outputs(self, h2):
        rows = h2.shape[0]
        s = self.scale_hid.fwd(h2, rows)
        mu = self.mean.fwd(s, rows)
        sr = self.std.fwd(s, rows)
        return s, mu, sr

    def _fused_args(self, g: GraphBatch):
        """dgppo_policy_step_args with this net's parameter pointers (None if the fused kernel does not
        cover the configuration)."""
        if os.environ.get("DGPPO_FUSED_POLICY", "1") != "1" or len(self.gnn.layers) > 2 or not self.gru.simple:
            return None  # (the fused kernel holds at most 2 GNN layers and one GRU layer; else the layer chain)
        a = _lib.PolicyStepArgs()
        a.N, a.E, a.n_agents, a.C, a.D0, a.A = g.N, g.E, self.n, g.C, g.nodes.shape[2], self.A
        a.n_layers, a.H, a.ED = len(self.gnn.layers), 3, g.ED
        for i, L in enumerate(self.gnn.layers):
            ly = a.layer[i]
            ly.Wq, ly.bq, ly.Wkt, ly.bk = K._p(L.v("Wq")), K._p(L.v("bq")), K._p(L.v("Wkt")), K._p(L.v("bk"))
            ly.Wcat, ly.Wu, ly.bu = K._p(L.v("Wcat")), K._p(L.v("Wu")), K._p(L.v("bu"))
            ly.Wex = K._p(L.v("Wex")) if getattr(L, "EX", 0) > 0 else None
            ly.D, ly.F = L.D, L.F
        hd = self.head
        a.head_W0, a.head_b0, a.head_W1, a.head_b1 = K._p(hd.d0.W()), K._p(hd.d0.b()), K._p(hd.d1.W()), K._p(hd.d1.b())
        a.ln0_s, a.ln0_b = K._p(self.ps.view(hd.ln0.name + ".scale")), K._p(self.ps.view(hd.ln0.name + ".bias"))
        a.ln1_s, a.ln1_b = K._p(self.ps.view(hd.ln1.name + ".scale")), K._p(self.ps.view(hd.ln1.name + ".bias"))
        gru = self.gru.cells[0]
        a.gru_Wi, a.gru_bi = K._p(gru.v("Wi")), K._p(gru.v("bi"))
        a.gru_Wh, a.gru_bhn = K._p(gru.v("Wh")), K._p(gru.v("bhn"))
        a.Ws, a.bs = K._p(self.scale_hid.W()), K._p(self.scale_hid.b())
        a.Wm, a.bm, a.Wsd, a.bsd = K._p(self.mean.W()), K._p(self.mean.b()), K._p(self.std.W()), K._p(self.std.b())
        a.std_shift, a.std_min = STD_DEV_INIT_INV, STD_DEV_MIN
        if not _lib.load().dgppo_policy_step_supported(ctypes.byref(a)):
            return None
        if getattr(self, "_policy_work", None) is None:
            self._policy_work = torch.zeros(_lib.load().dgppo_policy_work_floats(), device=self.ps.flat.device)
        a.work = K._p(self._policy_work)
        return a

    def act(self, g: GraphBatch, h: torch.Tensor, mode: int, noise=None, action_out=None, log_pi_out=None,
            h_out=None, prepare=True, noise_seed=None, noise_stream=0):
        """One policy step for G graphs: mode 0 = deterministic (get_action: tanh(mean)),
        1 = sample_action with standard-normal `noise` (G*n, A).  Returns (action, log_pi, h_new).
        Runs the fused dgppo_policy_step kernel when it covers the configuration; `prepare` refreshes
        its query-key products from the current weights (needed once after every weight change).
        noise_seed (a uint64 device scalar) + noise_stream: the noise is the Philox stream K.normal_ would write
        into `noise` -- drawn inside the fused kernel (no separate launch), else written to `noise` first."""
        rows = g.G * self.n
        fa = self._fused_args(g)
        if noise_seed is not None and mode == 1 and fa is None:
            K.normal_(noise, stream_id=noise_stream, seed_tensor=noise_seed)
        if fa is not None:
            if prepare:
                K._chk(_lib.load().dgppo_policy_prepare(ctypes.byref(fa), _lib.stream_handle(h.device)),
                       "dgppo_policy_prepare")
            dev = h.device
            h2 = h_out if h_out is not None else torch.empty_like(h)
            action = action_out if action_out is not None else torch.empty((rows, self.A), device=dev)
            log_pi = log_pi_out if log_pi_out is not None else torch.empty(rows, device=dev)
            fa.G, fa.mode = g.G, int(mode)
            fa.cand, fa.receivers, fa.senders = K._p(g.cand), K._p(g.receivers), K._p(g.senders)
            fa.nodes, fa.nodes_gstride = K._p(g.nodes), g.N * g.nodes.shape[2]
            fa.edges, fa.edges_gstride, fa.idx_gstride = K._p(g.edges), g.E * g.ED, g.E
            fa.h_in, fa.h_out = K._p(h), K._p(h2)
            if noise_seed is not None and mode == 1:  # ABI 10: drawn in the kernel
                fa.noise, fa.noise_seed, fa.noise_stream = None, K._p(noise_seed), int(noise_stream)
            else:
                fa.noise, fa.noise_seed, fa.noise_stream = K._p(noise), None, 0
            fa.action, fa.log_pi = K._p(action), K._p(log_pi)
            K._chk(_lib.load().dgppo_policy_step(ctypes.byref(fa), _lib.stream_handle(dev)), "dgppo_policy_step")
            return action, log_pi, h2
        y, _ = self._trunk(g, keep=False)
        feat, h2, _ = self.gru.fwd(y, h, h_out=h_out)
        _, mu, sr = self._outputs(feat)
        action = action_out if action_out is not None else torch.empty((rows, self.A), device=h.device)
        log_pi = log_pi_out if log_pi_out is not None else torch.empty(rows, device=h.device)
        a = _lib.TanhNormalArgs()
        a.rows, a.A, a.mode, a.n_agents = rows, self.A, mode, self.n
        a.mean, a.std_raw = K._p(mu), K._p(sr)
        a.std_shift, a.std_min = STD_DEV_INIT_INV, STD_DEV_MIN
        a.noise = K._p(noise)
        a.action_out, a.log_pi = K._p(action), K._p(log_pi)
        K.tanh_normal(a, h.device)
        return action, log_pi, h2

    def eval_seq_fwd(self, g: GraphBatch, S: int, L: int, actions: torch.Tensor, entropy_eps: torch.Tensor):
        """eval_action over S sequences of L steps (scan_eval_action, informarl.py:387-403), zero
        initial carries.  actions (S*L*n, A) rows (s, t, agent).  Returns log_pi, entropy (S*L*n,)."""
        n, dev = self.n, actions.device
        y, tc = self._trunk(g)  # (S*L*n, 64) rows (s, t, agent)
        H2, gcs = self.gru.seq_fwd(y, S * n, L, n)
        s, mu, sr = self._outputs(H2)
        rows = S * L * n
        log_pi = torch.empty(rows, device=dev)
        ent = torch.empty(rows, device=dev)
        a = _lib.TanhNormalArgs()
        a.rows, a.A, a.mode, a.n_agents = rows, self.A, 2, n
        a.mean, a.std_raw, a.action = K._p(mu), K._p(sr), K._p(actions)
        a.std_shift, a.std_min = STD_DEV_INIT_INV, STD_DEV_MIN
        a.log_pi, a.entropy, a.entropy_eps = K._p(log_pi), K._p(ent), K._p(entropy_eps)
        K.tanh_normal(a, dev)
        cache = (g, S, L, tc, gcs, H2, s, mu, sr, actions, entropy_eps)
        return log_pi, ent, cache

    def eval_seq_bwd(self, cache, dlog_pi, dentropy):
        g, S, L, tc, gcs, H2, s, mu, sr, actions, entropy_eps = cache
        n, dev = self.n, dlog_pi.device
        rows = S * L * n
        dmu = torch.empty_like(mu)
        dsr = torch.empty_like(sr)
        a = _lib.TanhNormalArgs()
        a.rows, a.A, a.mode, a.n_agents = rows, self.A, 2, n
        a.mean, a.std_raw, a.action = K._p(mu), K._p(sr), K._p(actions)
        a.std_shift, a.std_min = STD_DEV_INIT_INV, STD_DEV_MIN
        a.entropy_eps = K._p(entropy_eps)
        a.dlog_pi, a.dentropy, a.dmean, a.dstd_raw = K._p(dlog_pi), K._p(dentropy), K._p(dmu), K._p(dsr)
        K.tanh_normal(a, dev)
        ds = self.mean.bwd(s, dmu, rows)
        self.std.bwd(s, dsr, rows, dx_out=ds, accumulate=True)
        dH2 = self.scale_hid.bwd(H2, ds, rows)
        self._bptt(dH2.view(S, L, n, 64), gcs, S, L, tc, g)

    def _bptt(self, dHs, gcs, S, L, tc, g):
        gc, hc = tc
        ln = self.head.ln1_bwd_args(hc) if self.gru.simple else None  # LayerNorm_1 bwd in the GRU's dx GEMM
        dY, _ = self.gru.seq_bwd(gcs, dHs.reshape(S * L * self.n, 64), ln=ln)
        fused = ln is not None
        dz = self.head.bwd(hc, dY, dy_is_dh1=fused, mask_input=fused)
        self.gnn.bwd(gc, dz, g, top_masked=fused)


class VlNet(_Net):
    def __init__(self, node_dim: int, n_agents: int, device, seed: int = 1, gnn_layers: int = 2, edge_dim: int = 4,
                 rnn: str = "gru", rnn_layers: int = 1):
        self.n = n_agents
        ps = self.ps = ParamSpace()
        self.gnn = GNN(ps, "gnn", node_dim, gnn_layers, edge_dim=edge_dim)
        self.head = MLPHead(ps, "head")
        self.gru = RNNStack(ps, "gru", rnn, rnn_layers)  # RNN(GRUCell | LSTMCell, layers) or none
        self.out = Dense(ps, "out", 64, 1)
        self.modules = [self.gnn, self.head, self.gru, self.out]
        ps.build(device)
        self.init_host(seed)
        self.device = torch.device(device)

    def flax(self):
        return {"gnn": self.gnn.flax(), "head": self.head.flax(), "gru": self.gru.flax(), "out": self.out.flax()}

    def load_flax(self, d):
        self.gnn.load_flax(d["gnn"]), self.head.load_flax(d["head"]), self.gru.load_flax(d["gru"])
        self.out.load_flax(d["out"])

    def graph_means(self, g: GraphBatch, out=None):
        """The GNN part of the value: the agent mean of the last GNN layer's agent rows, (G, 64) (graphs are
        independent here; seq_fwd's sequence structure starts after it)."""
        zm = out if out is not None else torch.empty((g.G, 64), device=g.nodes.device)
        if self.gnn.fwd_epilogue(g, zmean=zm) is not None:  # the mean in the last layer's kernel (Y never stored)
            return zm
        z, _ = self.gnn.fwd(g, keep=False)
        K.agent_mean_fwd(z, zm, g.G, self.n, 64, self.n * 64)
        return zm

    def seq_fwd(self, g: GraphBatch, S: int, L: int, h0=None, keep_cache=True, zm=None):
        """scan_Vl (informarl.py:281-293) over S sequences of L graphs.  Returns values (S, L),
        final carries (S, 64) and the cache for seq_bwd.  zm: the graphs' agent means already computed
        (graph_means, rows s * L + t; forward only, g unused)."""
        dev = self.ps.flat.device
        G = S * L
        if zm is not None:
            assert not keep_cache, "seq_fwd from precomputed agent means is forward-only"
            z = gc = None
        else:
            n = self.n
            z, gc = self.gnn.fwd(g, keep=keep_cache)  # (G*n, 64)
            zm = torch.empty((G, 64), device=dev)
            K.agent_mean_fwd(z, zm, G, n, 64, n * 64)
        y, hc = self.head.fwd(zm)
        hT = torch.empty((S, self.gru.W), device=dev)
        Hs, gcs = self.gru.seq_fwd(y, S, L, 1, h0=h0, hT_out=hT)
        v = self.out.fwd(Hs, G)
        cache = (g, S, L, gc, z, hc, gcs, Hs) if keep_cache else None
        return v.view(S, L), hT, cache

    def seq_bwd(self, cache, dv):
        g, S, L, gc, z, hc, gcs, Hs = cache
        n, dev = self.n, dv.device
        G = S * L
        dH = self.out.bwd(Hs, dv.reshape(G, 1).contiguous(), G)
        ln = self.head.ln1_bwd_args(hc) if self.gru.simple else None
        dY, _ = self.gru.seq_bwd(gcs, dH, ln=ln)
        dzm = self.head.bwd(hc, dY, dy_is_dh1=ln is not None)
        dz = torch.empty_like(z)
        # z is the last GNN layer's ReLU output: its gate is fused into the broadcast (FUSE_LN, as the GEMM epilogues)
        K.agent_mean_bwd(dzm, dz, G, n, 64, n * 64, mask=z if FUSE_LN else None)
        self.gnn.bwd(gc, dz, g, top_masked=FUSE_LN)


class VhNet(_Net):
    def __init__(self, node_dim: int, n_agents: int, n_cost: int, device, seed: int = 2, gnn_layers: int = 1,
                 edge_dim: int = 4, rnn: str = "gru", rnn_layers: int = 1):
        self.n, self.n_cost = n_agents, n_cost
        ps = self.ps = ParamSpace()
        self.gnn = GNN(ps, "gnn", node_dim, gnn_layers, edge_dim=edge_dim)
        self.head = MLPHead(ps, "head")
        self.gru = RNNStack(ps, "gru", rnn, rnn_layers)  # RNN(GRUCell | LSTMCell, layers) or none
        self.out = Dense(ps, "out", 64, n_cost)
        self.modules = [self.gnn, self.head, self.gru, self.out]
        ps.build(device)
        self.init_host(seed)
        self.device = torch.device(device)

    def flax(self):
        return {"gnn": self.gnn.flax(), "head": self.head.flax(), "gru": self.gru.flax(), "out": self.out.flax()}

    def load_flax(self, d):
        self.gnn.load_flax(d["gnn"]), self.head.load_flax(d["head"]), self.gru.load_flax(d["gru"])
        self.out.load_flax(d["out"])

    def fwd(self, g: GraphBatch, h: torch.Tensor, keep_cache=True):
        """get_Vh (dgppo.py:128-134) on G graphs with the actor's carries h (G*n, W): (G*n, n_cost).  Forward only
        (keep_cache False): GNN, head, GRU step and output Dense in one kernel where it applies (the prepass)."""
        rows = g.G * self.n
        self.last_tail = False  # True when the fused kernel's value-head tail produced the output (tests)
        if VH_TAIL and not keep_cache and self.gru.simple and len(self.gnn.layers) == 1 and h.shape[1] == 64:
            out = torch.empty((rows, self.n_cost), device=h.device)
            hd, cell = self.head, self.gru.cells[0]
            v = self.ps.view
            tail_w = [hd.d0.W(), hd.d0.b(), v(hd.ln0.name + ".scale"), v(hd.ln0.name + ".bias"), hd.d1.W(), hd.d1.b(),
                      v(hd.ln1.name + ".scale"), v(hd.ln1.name + ".bias"), cell.v("Wi"), cell.v("bi"), cell.v("Wh"),
                      cell.v("bhn"), self.out.W(), self.out.b()]
            if self.gnn.fwd_epilogue(g, tail=(tail_w, h if h.is_contiguous() else h.contiguous(), out)) is not None:
                self.last_tail = True
                return out, None
        z, gc = self.gnn.fwd(g, keep=keep_cache)
        y, hc = self.head.fwd(z)
        h2, _, rc = self.gru.fwd(y, h)
        out = self.out.fwd(h2, rows)
        return out, ((g, gc, hc, rc, h2) if keep_cache else None)

    def bwd(self, cache, dout):
        g, gc, hc, rc, h2 = cache
        rows = g.G * self.n
        dh2 = self.out.bwd(h2, dout, rows)
        ln = self.head.ln1_bwd_args(hc) if self.gru.simple else None
        dy, _ = self.gru.seq_bwd(rc, dh2, ln=ln)
        fused = ln is not None
        dz = self.head.bwd(hc, dy, dy_is_dh1=fused, mask_input=fused)
        self.gnn.bwd(gc, dz, g, top_masked=fused)


class VhGlobalNet(_Net):
    """InforMARL-Lagr's cost critic: ValueNet(n_out=n_cost, decompose=True, use_global_info=True)
    (DecRStateFn, value.py:47-79; informarl_lagr.py:68-79): GNN(agent rows) -> [x | mean over agents of x]
    (n, 128) -> MLP(64, 64) -> GRUCell with its OWN carries (scan_Vh, informarl_lagr.py:152-163) ->
    Dense(n_cost).  The concat never materialises: head Dense_0 = x W[:64] + b + broadcast(mean(x) W[64:])
    (one GEMM of the agent-mean rows, added per graph through the GEMM addend's row grouping)."""

    def __init__(self, node_dim: int, n_agents: int, n_cost: int, device, seed: int = 2, gnn_layers: int = 1,
                 edge_dim: int = 4, rnn: str = "gru", rnn_layers: int = 1):
        self.n, self.n_cost = n_agents, n_cost
        ps = self.ps = ParamSpace()
        self.gnn = GNN(ps, "gnn", node_dim, gnn_layers, edge_dim=edge_dim)
        self.head = MLPHead(ps, "head", d_in=128)
        self.gru = RNNStack(ps, "gru", rnn, rnn_layers)  # RNN(GRUCell | LSTMCell, layers) or none
        self.out = Dense(ps, "out", 64, n_cost)
        self.modules = [self.gnn, self.head, self.gru, self.out]
        ps.build(device)
        self.init_host(seed)
        self.device = torch.device(device)

    def flax(self):
        return {"gnn": self.gnn.flax(), "head": self.head.flax(), "gru": self.gru.flax(), "out": self.out.flax()}

    def load_flax(self, d):
        self.gnn.load_flax(d["gnn"]), self.head.load_flax(d["head"]), self.gru.load_flax(d["gru"])
        self.out.load_flax(d["out"])

    def seq_fwd(self, g: GraphBatch, S: int, L: int, h0=None, keep_cache=True):
        """scan_Vh over S sequences of L graphs (zero carries unless h0 (S*n, 64)): values (S*L*n, n_cost) rows
        (s, t, agent), final carries (S*n, 64) and the cache for seq_bwd."""
        n, dev = self.n, g.nodes.device
        G = S * L
        rows = G * n
        z, gc = self.gnn.fwd(g, keep=keep_cache)  # (rows, 64)
        zm = torch.empty((G, 64), device=dev)
        K.agent_mean_fwd(z, zm, G, n, 64, n * 64)
        W0 = self.head.d0.W()
        m = torch.empty((G, 64), device=dev)
        K.gemm(zm, W0[64:], m, G, 64, 64)
        h0pre = torch.empty((rows, 64), device=dev)
        K.gemm(z, W0[:64], h0pre, rows, 64, 64, bias=self.head.d0.b(), addend=m, ld_add=0, add_grp=n, add_gs=64)
        hd = self.head
        y0, c0 = hd.ln0.fwd(h0pre)
        h1 = hd.d1.fwd(y0, rows)
        y1, c1 = hd.ln1.fwd(h1)
        hT = torch.empty((S * n, self.gru.W), device=dev)
        Hs, gcs = self.gru.seq_fwd(y1, S * n, L, n, h0=h0, hT_out=hT)
        out = self.out.fwd(Hs, rows)
        cache = (g, S, L, gc, z, zm, y0, c0, c1, gcs, Hs) if keep_cache else None
        return out, hT, cache

    def seq_bwd(self, cache, dout):
        g, S, L, gc, z, zm, y0, c0, c1, gcs, Hs = cache
        n, dev = self.n, dout.device
        G = S * L
        rows = G * n
        hd = self.head
        dH = self.out.bwd(Hs, dout, rows)
        dy1, _ = self.gru.seq_bwd(gcs, dH)
        dh1 = hd.ln1.bwd(c1, dy1)
        dy0 = hd.d1.bwd(y0, dh1, rows)
        dh0 = hd.ln0.bwd(c0, dy0)  # d(head Dense_0 output) (rows, 64)
        W0, dW0 = hd.d0.W(), hd.d0.W(True)
        K.gemm(z, dh0, dW0[:64], 64, 64, rows, ta=True, beta=1.0, bias_grad=hd.d0.b(True))
        sm = torch.empty((G, 64), device=dev)  # per-graph mean of dh0; the agent SUM is n x it
        K.agent_mean_fwd(dh0, sm, G, n, 64, n * 64)
        K.gemm(zm, sm, dW0[64:], 64, 64, G, ta=True, alpha=float(n), beta=1.0)
        # dz = dh0 W[:64]^T + (sum_agents dh0) W[64:]^T / n  (the mean's backward), one GEMM with a per-graph addend
        dzm = torch.empty((G, 64), device=dev)
        K.gemm(sm, W0[64:], dzm, G, 64, 64, tb=True, ldb=64)
        dz = torch.empty_like(z)
        K.gemm(dh0, W0[:64], dz, rows, 64, 64, tb=True, ldb=64, addend=dzm, ld_add=0, add_grp=n, add_gs=64)
        self.gnn.bwd(gc, dz, g)

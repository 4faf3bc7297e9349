"""Typed wrappers over the hot-path-(2) C-ABI (include/dgppo_hip.h) for torch device tensors (the
registered torch.ops.dgppo ops where one exists, dgppo_fov_amd/ops.py).

Every function launches on torch's current stream and returns immediately; there is no CPU
path (non-CUDA tensors raise NativeLibraryError)."""
from __future__ import annotations

import ctypes
import math
import weakref

import torch

from .. import _lib, ops  # noqa: F401  (ops registers torch.ops.dgppo.*)

_WS = {}
_GRAPHS = weakref.WeakSet()  # captured hipGraphs still alive (registered by hold_for_graph before their capture)
_WS_KEPT = []  # (replaced workspace buffer, weak references to the graphs alive when it was replaced)


def hold_for_graph(g):
    """Register a hipGraph (torch.cuda.CUDAGraph) BEFORE its capture starts: until it is garbage-collected, a
    workspace buffer that is replaced by a larger one stays allocated, because the graph's kernels keep its
    address (a replay would otherwise write into memory the allocator has handed to another tensor)."""
    _GRAPHS.add(g)
    return g


def workspace(nfloats: int, device, slot: str = "default") -> torch.Tensor:
    """Grow-only scratch buffer per (device, slot, current stream): reused by the sequential launches of
    one stream, never shared by launches that may run concurrently on different streams."""
    key = (str(device), slot, _lib.stream_handle(device))
    t = _WS.get(key)
    if t is None or t.numel() < nfloats:
        old = t.numel() if t is not None else 0
        live = [weakref.ref(g) for g in _GRAPHS]
        if t is not None and live:
            _WS_KEPT.append((t, live))  # a live graph may hold its address: freed once every such graph is gone
        _WS_KEPT[:] = [(b, refs) for b, refs in _WS_KEPT if any(r() is not None for r in refs)]
        # with graphs alive growth doubles, so the kept buffers stay below the final size; otherwise exact
        t = torch.empty(max(int(nfloats), 2 * old if live else 0, 1024), dtype=torch.float32, device=device)
        _WS[key] = t
    return t


def _p(t, off=0):
    return 0 if t is None else int(t.data_ptr()) + 4 * int(off)


def _stream(t):
    return _lib.stream_handle(t.device)


def _chk(rc, what):
    _lib.check(rc, what)


GEMM_LOG = None  # set to a list to record (M, N, K, batch, ta, tb, split_k, has_bias) per launch

# weight-gradient GEMMs deferred to the end of a network pass's backward (defer_wgrad): current stream handle ->
# [(GemmArgs copy, tensors held until the launch, (C start, C end), (bias start, bias end))]
_DEFER = {}
_DEFER_GRADS = {}  # stream handle -> [start, end) bytes of the parameter-gradient buffer deferred outputs must lie in
DEFER_MAX = 64  # pending problems per stream before an early flush


def _extent(t_ptr, rows, cols, ld, grp, gstride, batch=1, bstride=0):
    """[start, end) byte range of a (rows, cols) float matrix at address t_ptr with row grouping (grp rows per group,
    gstride floats between groups) and batch entries bstride floats apart."""
    if rows <= 0 or cols <= 0:
        return (t_ptr, t_ptr)
    if grp > 0:
        last = ((rows - 1) // grp) * gstride + (min(grp, rows) - 1) * ld
    else:
        last = (rows - 1) * ld
    return (t_ptr, t_ptr + 4 * ((batch - 1) * bstride + last + cols))


def _in_workspace(ptr, device) -> bool:
    dev = str(device)
    for (d, _, _), t in _WS.items():
        if d == dev and t.data_ptr() <= ptr < t.data_ptr() + 4 * t.numel():
            return True
    for t, _ in _WS_KEPT:
        if t.device == device and t.data_ptr() <= ptr < t.data_ptr() + 4 * t.numel():
            return True
    return False


class defer_wgrad:
    """Inside this context the weight-gradient GEMMs (gemm(..., ta=True) on the wgrad path) issued on the current
    stream whose outputs (C and bias_grad) lie in `grads` -- the pass's parameter-gradient buffer -- are recorded
    instead of launched, and launched together on exit: ONE grouped kernel + ONE partial reduction per 12 problems
    (dgppo_gemm_wgrad_grouped, ABI 13) instead of two launches each, every output bit-identical.  Safe because
    nothing reads a parameter gradient before the pass ends (a wgrad GEMM into a temporary, e.g. the Q-free
    projections' [x 1]^T [dqt | dbeta] that the next GEMM reads, runs at once) and the recorded inputs are held (a
    call whose A / B lives in a workspace slot, which later launches reuse, runs at once; one whose C / bias_grad
    overlaps a pending problem's first flushes the pending ones, keeping the accumulation order).  on=False: a
    no-op."""

    def __init__(self, device, grads=None, on=True):
        self.device, self.on = device, on and grads is not None and torch.device(device).type == "cuda"
        self.grads = grads

    def __enter__(self):
        if self.on:
            self.key = _lib.stream_handle(self.device)
            self.prev = _DEFER.get(self.key)
            _DEFER[self.key] = []
            g = self.grads
            _DEFER_GRADS[self.key] = (g.data_ptr(), g.data_ptr() + 4 * g.numel())
        return self

    def __exit__(self, *exc):
        if self.on:
            try:
                if exc[0] is None:
                    flush_wgrad(self.device, self.key)
            finally:
                _DEFER_GRADS.pop(self.key, None)
                if self.prev is None:
                    _DEFER.pop(self.key, None)
                else:
                    _DEFER[self.key] = self.prev
        return False


def flush_wgrad(device, key=None):
    key = _lib.stream_handle(device) if key is None else key
    pend = _DEFER.get(key)
    if not pend:
        return
    lib = _lib.load()
    n = len(pend)
    arr = (_lib.GemmArgs * n)(*[e[0] for e in pend])
    nws = lib.dgppo_gemm_wgrad_grouped_workspace_floats(arr, n)
    ws = _p(workspace(nws, device, "wgrad_group")) if nws > 0 else None
    _chk(lib.dgppo_gemm_wgrad_grouped(arr, n, ws, _lib.stream_handle(device)), "dgppo_gemm_wgrad_grouped")
    pend.clear()


def _try_defer(g, A, B, C, bias_grad, relu, bias, addend, mask, ln) -> bool:
    """Record a weight-gradient GEMM in the current stream's defer_wgrad list (True) or leave it to run now."""
    if not _DEFER or not (g.trans_a and not g.trans_b) or bias is not None or addend is not None or relu or \
            mask is not None or ln is not None or g.N > 192 or g.M > 4096 or g.M < 1 or g.N < 1:
        return False
    key = _lib.stream_handle(C.device)
    pend = _DEFER.get(key)
    if pend is None or _in_workspace(g.A, C.device) or _in_workspace(g.B, C.device):
        return False
    cr = _extent(g.C, g.M, g.N, g.ldc, g.c_grp, g.c_gstride, g.batch, g.stride_c)
    br = (g.bias_grad, g.bias_grad + 4 * g.N * g.batch) if g.bias_grad else (0, 0)
    lo, hi = _DEFER_GRADS[key]
    if not (lo <= cr[0] and cr[1] <= hi and (br[0] == br[1] or (lo <= br[0] and br[1] <= hi))):
        return False  # not a parameter gradient: something later in the pass may read it
    for _, _, c2, b2 in pend:
        if any(x[0] < y[1] and y[0] < x[1] for x in (cr, br) for y in (c2, b2) if x[0] != x[1] and y[0] != y[1]):
            flush_wgrad(C.device)  # (the overlapping accumulation keeps its order)
            break
    if len(pend) >= DEFER_MAX:
        flush_wgrad(C.device)
    pend.append((type(g).from_buffer_copy(g), (A, B, C, bias_grad), cr, br))
    return True

def gemm(A, B, C, M, N, K, *, ta=False, tb=False, lda=None, ldb=None, ldc=None, batch=1, sa=0, sb=0, sc=0,
         a_off=0, b_off=0, c_off=0, a_grp=0, a_gs=0, b_grp=0, b_gs=0, c_grp=0, c_gs=0,
         bias=None, addend=None, add_off=0, ld_add=None, add_grp=0, add_gs=0,
         alpha=1.0, beta=0.0, relu=False, split_k=None, bias_grad=None, mask=None, ld_mask=None, ln=None):
    """C = alpha op(A) op(B) + beta C + bias + addend (see dgppo_gemm).  Element offsets/strides.
    bias_grad (ta only): bias_grad = alpha colsum(B) + beta bias_grad, fused into the dW GEMM.
    mask: C = mask > 0 ? result : 0 (the ReLU backward fused into the epilogue, ABI 9 epi 1).
    ln: LayerNorm(64) + ReLU epilogue (epi 2 / 3): dict(mode="fwd" | "bwd", scale, bias, h, mean, rstd,
    dscale, dbias) -- fwd writes h (pre-LN rows), mean, rstd and C = y; bwd reads h, mean, rstd, writes C = dx and
    accumulates dscale / dbias (per-workgroup partials summed by dgppo_colsum)."""
    lib = _lib.load()
    _lib.require_gpu(C.device, "gemm")
    g = _lib.GemmArgs()
    g.M, g.N, g.K, g.batch = int(M), int(N), int(K), int(batch)
    g.trans_a, g.trans_b = int(ta), int(tb)
    g.A, g.lda, g.stride_a = _p(A, a_off), int(lda if lda is not None else (M if ta else K)), int(sa)
    g.B, g.ldb, g.stride_b = _p(B, b_off), int(ldb if ldb is not None else (K if tb else N)), int(sb)
    g.C, g.ldc, g.stride_c = _p(C, c_off), int(ldc if ldc is not None else N), int(sc)
    g.a_grp, g.b_grp, g.c_grp = int(a_grp), int(b_grp), int(c_grp)
    g.a_gstride, g.b_gstride, g.c_gstride = int(a_gs), int(b_gs), int(c_gs)
    g.bias = _p(bias)
    g.addend, g.ld_add, g.stride_add = _p(addend, add_off), int(ld_add if ld_add is not None else N), 0
    g.add_grp, g.add_gstride = int(add_grp), int(add_gs)
    g.alpha, g.beta, g.relu = float(alpha), float(beta), int(relu)
    if split_k is None:
        tiles = math.ceil(M / 64) * math.ceil(N / 64) * batch
        split_k = max(1, min(math.ceil(K / 512), 1024 // max(tiles, 1))) if K >= 2048 else 1
    g.split_k = int(split_k)
    g.bias_grad = _p(bias_grad)
    part = None
    if mask is not None:
        g.epi, g.mask, g.ld_mask = 1, _p(mask), int(ld_mask if ld_mask is not None else N)
    if ln is not None:
        g.epi = 2 if ln["mode"] == "fwd" else 3
        g.ln_scale, g.ln_bias, g.ln_h = _p(ln["scale"]), _p(ln["bias"]), _p(ln["h"])
        g.ln_mean, g.ln_rstd = _p(ln["mean"]), _p(ln["rstd"])  # fwd writes them, bwd reads the fwd's
        if g.epi == 3:
            nrow = _lib.load().dgppo_gemm_partial_rows(ctypes.byref(g))
            part = workspace(nrow * 128, C.device, "gemm_ln_part")
            g.ln_part = _p(part)
    if GEMM_LOG is not None:
        GEMM_LOG.append((int(M), int(N), int(K), int(batch), int(ta), int(tb), int(split_k), bias is not None))
    if _DEFER and _try_defer(g, A, B, C, bias_grad, relu, bias, addend, mask, ln):
        return
    nws = lib.dgppo_gemm_workspace_floats(ctypes.byref(g))
    g.workspace = _p(workspace(nws, C.device, "gemm")) if nws > 0 else None
    _chk(lib.dgppo_gemm(ctypes.byref(g), _stream(C)), "dgppo_gemm")
    if part is not None:  # [dscale | dbias] partial rows -> += the LayerNorm parameter gradients
        ds, db = ln["dscale"], ln["dbias"]
        if db.data_ptr() == ds.data_ptr() + 4 * 64:  # adjacent in the flat gradient buffer: one reduction
            colsum(part, nrow, 128, ds, beta=1.0)  # writes ds[0:64] and the dbias that follows
        else:
            colsum(part, nrow, 64, ds, ld=128, beta=1.0)
            colsum(part, nrow, 64, db, ld=128, x_off=64, beta=1.0)


def colsum(x, rows, cols, out, *, ld=None, grp=0, gs=0, x_off=0, alpha=1.0, beta=0.0):
    lib = _lib.load()
    ws = workspace(lib.dgppo_colsum_workspace_floats(int(rows), int(cols)), out.device, "colsum")
    _chk(lib.dgppo_colsum(_p(x, x_off), int(rows), int(cols), int(ld if ld is not None else cols), int(grp), int(gs),
                          _p(out), float(alpha), float(beta), _p(ws), _stream(out)), "dgppo_colsum")


def relu_bwd_(dy, y):
    _chk(_lib.load().dgppo_relu_bwd(_p(dy), _p(y), int(dy.numel()), _stream(dy)), "dgppo_relu_bwd")


def lstm_cell_fwd(rows, H, g, c_prev, c_out, h_out):
    _chk(_lib.load().dgppo_lstm_cell_fwd(int(rows), int(H), _p(g), _p(c_prev), _p(c_out), _p(h_out), _stream(g)),
         "dgppo_lstm_cell_fwd")


def lstm_cell_bwd(rows, H, g, c_prev, c, dh, dc, dg, dc_prev):
    _chk(_lib.load().dgppo_lstm_cell_bwd(int(rows), int(H), _p(g), _p(c_prev), _p(c), _p(dh), _p(dc), _p(dg),
                                         _p(dc_prev), _stream(g)), "dgppo_lstm_cell_bwd")


def layernorm_fwd(x, scale, bias, y, mean, rstd, relu=True, eps=1e-6):
    rows, F = x.shape
    _chk(_lib.load().dgppo_layernorm_fwd(_p(x), _p(scale), _p(bias), _p(y), _p(mean), _p(rstd), int(rows), int(F),
                                         int(relu), float(eps), _stream(x)), "dgppo_layernorm_fwd")


def layernorm_bwd(x, y, dy, scale, mean, rstd, dx, dscale, dbias, relu=True):
    lib = _lib.load()
    rows, F = x.shape
    ws = workspace(lib.dgppo_layernorm_bwd_workspace_floats(int(rows), int(F)), x.device, "ln")
    _chk(lib.dgppo_layernorm_bwd(_p(x), _p(y), _p(dy), _p(scale), _p(mean), _p(rstd), _p(dx), _p(dscale), _p(dbias),
                                 int(rows), int(F), int(relu), _p(ws), _stream(x)), "dgppo_layernorm_bwd")


def gru_fwd(gi, gh, bhn, h, h_new):
    rows, H = h.shape
    _chk(_lib.load().dgppo_gru_fwd(_p(gi), _p(gh), _p(bhn), _p(h), _p(h_new), int(rows), int(H), _stream(h)),
         "dgppo_gru_fwd")


def gru_bwd(gi, gh, bhn, h, dh_new, dgi, dgh, dh):
    rows, H = h.shape
    _chk(_lib.load().dgppo_gru_bwd(_p(gi), _p(gh), _p(bhn), _p(h), _p(dh_new), _p(dgi), _p(dgh), _p(dh), int(rows),
                                   int(H), _stream(h)), "dgppo_gru_bwd")


def gru_seq(fwd, Q, L, n, gi, Wh, bhn, h0, hs, hT=None, dhs=None, dgi=None, dgh=None, dh0=None, dbhn_part=None):
    a = _lib.GruSeqArgs()
    a.Q, a.L, a.n_agents, a.H = int(Q), int(L), int(n), 64
    a.gi, a.Wh, a.bhn, a.h0, a.hs, a.hT = _p(gi), _p(Wh), _p(bhn), _p(h0), _p(hs), _p(hT)
    a.dhs, a.dgi, a.dgh, a.dh0, a.dbhn_part = _p(dhs), _p(dgi), _p(dgh), _p(dh0), _p(dbhn_part)
    lib = _lib.load()
    if fwd:
        _chk(lib.dgppo_gru_seq_fwd(ctypes.byref(a), _stream(hs)), "dgppo_gru_seq_fwd")
    else:
        _chk(lib.dgppo_gru_seq_bwd(ctypes.byref(a), _stream(hs)), "dgppo_gru_seq_bwd")


def gru_seq_blocks(Q):
    return int(_lib.load().dgppo_gru_seq_blocks(int(Q)))


def agent_mean_fwd(x, y, G, n, F, x_gstride):
    _chk(_lib.load().dgppo_agent_mean_fwd(_p(x), _p(y), int(G), int(n), int(F), int(x_gstride), _stream(y)),
         "dgppo_agent_mean_fwd")


def agent_mean_bwd(dy, dx, G, n, F, dx_gstride, mask=None):
    """dx = broadcast(dy) / n over each graph's n agent rows; mask: the ReLU output rows (G n, F) that fed the mean,
    dx = mask > 0 ? dy / n : 0 (its ReLU backward fused)."""
    _chk(_lib.load().dgppo_agent_mean_bwd_masked(_p(dy), _p(mask), _p(dx), int(G), int(n), int(F), int(dx_gstride),
                                                 _stream(dx)), "dgppo_agent_mean_bwd_masked")


def sender_table(G, n, C, E, cand, receivers, senders, out):
    _chk(_lib.load().dgppo_gnn_sender_table(int(G), int(n), int(C), int(E), _p(cand), _p(receivers), _p(senders),
                                            _p(out), _stream(out)), "dgppo_gnn_sender_table")


def edge_wsum(G, n, C, H, EX, E, attn, cand, sidx, efx, out):
    _chk(_lib.load().dgppo_gnn_edge_wsum(int(G), int(n), int(C), int(H), int(EX), int(E), _p(attn), _p(cand),
                                         _p(sidx), _p(efx), _p(out), _stream(out)), "dgppo_gnn_edge_wsum")


def edge_da(G, n, C, H, EX, E, dxx, cand, sidx, efx, out):
    _chk(_lib.load().dgppo_gnn_edge_da(int(G), int(n), int(C), int(H), int(EX), int(E), _p(dxx), _p(cand),
                                       _p(sidx), _p(efx), _p(out), _stream(out)), "dgppo_gnn_edge_da")


def tanh_normal(args: _lib.TanhNormalArgs, device):
    _chk(_lib.load().dgppo_tanh_normal(ctypes.byref(args), _lib.stream_handle(device)), "dgppo_tanh_normal")


def ppo_loss(log_pi, log_pi_old, adv, entropy, clip_eps, coef_ent, dlog_pi, dentropy, stats):
    lib = _lib.load()
    ws = workspace(lib.dgppo_loss_workspace_floats(), log_pi.device, "loss")
    _chk(lib.dgppo_ppo_loss(_p(log_pi), _p(log_pi_old), _p(adv), _p(entropy), int(log_pi.numel()), float(clip_eps),
                            float(coef_ent), _p(dlog_pi), _p(dentropy), _p(stats), _p(ws), _stream(log_pi)),
         "dgppo_ppo_loss")


def l2_loss(pred, target, dpred, loss):
    lib = _lib.load()
    ws = workspace(lib.dgppo_loss_workspace_floats(), pred.device, "loss")
    _chk(lib.dgppo_l2_loss(_p(pred), _p(target), int(pred.numel()), _p(dpred), _p(loss), _p(ws), _stream(pred)),
         "dgppo_l2_loss")


def gae(hs, l, Vh, Vl, Qh, Ql, gamma, lam):
    torch.ops.dgppo.gae(hs, l, Vh, Vl, Qh, Ql, float(gamma), float(lam))


def grad_norm(grad, state):
    torch.ops.dgppo.grad_norm(grad, state)


def adam(param, grad, m, v, state, lr, b1=0.9, b2=0.999, eps=1e-8, max_norm=2.0):
    torch.ops.dgppo.adam(param, grad, m, v, state, float(lr), float(b1), float(b2), float(eps), float(max_norm))


def adam_multi(nets, b1=0.9, b2=0.999, eps=1e-8):
    """grad_norm + adam (the pair above) for up to 4 nets in two launches, bit-identical to the per-net calls:
    nets = [(param, grad, m, v, state, lr, max_norm), ...] (dgppo_adam_multi, ABI 12)."""
    lib = _lib.load()
    a = _lib.AdamMultiArgs()
    a.n_nets, a.eps, a.b1, a.b2 = len(nets), float(eps), float(b1), float(b2)
    if not 1 <= len(nets) <= _lib.ADAM_MAX_NETS:
        raise ValueError(f"{len(nets)} nets (1..{_lib.ADAM_MAX_NETS})")
    param0 = nets[0][0]
    a.workspace = _p(workspace(lib.dgppo_adam_multi_workspace_floats(), param0.device, "adam_multi"))
    for k, (param, grad, m, v, state, lr, max_norm) in enumerate(nets):
        t = a.net[k]
        t.param, t.grad, t.m, t.v, t.state = _p(param), _p(grad), _p(m), _p(v), _p(state)
        t.n, t.lr, t.max_norm = int(param.numel()), float(lr), float(max_norm)
    _chk(lib.dgppo_adam_multi(ctypes.byref(a), _stream(param0)), "dgppo_adam_multi")


def normal_(out, seed=0, stream_id=0, seed_tensor=None):
    _chk(_lib.load().dgppo_normal(_p(out), int(out.numel()), _p(seed_tensor), int(seed) & 0xFFFFFFFFFFFFFFFF,
                                  int(stream_id) & 0xFFFFFFFFFFFFFFFF, _stream(out)), "dgppo_normal")
    return out


def cost_shaped_loss(rewards, costs, cost_weight, out):
    B, T, n, nh = costs.shape
    _chk(_lib.load().dgppo_cost_shaped_loss(_p(rewards), _p(costs), float(cost_weight), _p(out), int(B), int(T), int(n),
                                            int(nh), _stream(out)), "dgppo_cost_shaped_loss")


def informarl_advantages(Ql, Vl, A):
    B, T, n = A.shape
    _chk(_lib.load().dgppo_informarl_advantages(_p(Ql), _p(Vl), _p(A), int(B), int(T), int(n), _stream(A)),
         "dgppo_informarl_advantages")


def dgppo_advantages(Ql, Vl, Vh, A, safe_count, dt, alpha, cbf_eps, cbf_weight):
    B, T = Ql.shape
    _, _, n, nh = Vh.shape
    a = _lib.AdvArgs()
    a.B, a.T, a.n_agents, a.n_h = int(B), int(T), int(n), int(nh)
    a.Ql, a.Vl, a.Vh, a.A, a.safe_count = _p(Ql), _p(Vl), _p(Vh), _p(A), _p(safe_count)
    a.dt, a.alpha, a.cbf_eps, a.cbf_weight = float(dt), float(alpha), float(cbf_eps), float(cbf_weight)
    _chk(_lib.load().dgppo_dgppo_advantages(ctypes.byref(a), _stream(Ql)), "dgppo_dgppo_advantages")


def clip_min0(x, y):
    _chk(_lib.load().dgppo_clip_min0(_p(x), _p(y), int(x.numel()), _stream(y)), "dgppo_clip_min0")


def lagr_advantages(Ql, Vl, Qh, Vh, lagr, A, Ah):
    B, T, n, nh = Qh.shape
    _chk(_lib.load().dgppo_lagr_advantages(_p(Ql), _p(Vl), _p(Qh), _p(Vh), _p(lagr), _p(A), _p(Ah), int(B), int(T),
                                           int(n), int(nh), _stream(A)), "dgppo_lagr_advantages")


def lagr_update(log_pi, log_pi_old, Vh, Ah, lagr, lagr_mean, rows, gamma, lr):
    n, nh = lagr.shape
    _chk(_lib.load().dgppo_lagr_update(_p(log_pi), _p(log_pi_old), _p(Vh), _p(Ah), _p(lagr), _p(lagr_mean), int(rows),
                                       int(n), int(nh), float(gamma), float(lr), _stream(lagr)), "dgppo_lagr_update")

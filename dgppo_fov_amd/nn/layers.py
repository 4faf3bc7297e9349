"""Network layers of the DGPPO actor / critics with explicit forward and backward passes.

Counterparts of dgppo/nn/gnn.py (GraphTransformer, GraphTransformerGNN), dgppo/nn/mlp.py (MLP with
LayerNorm), dgppo/nn/rnn.py + flax GRUCell, and flax Dense.  Parameters of a network live in ONE
flat fp32 buffer (and gradients in a twin buffer), so gradient clipping, the finite check, Adam
and the multi-GPU all-reduce are single launches over contiguous memory.  All arithmetic runs in
libdgppo_hip.so (dgppo_gemm, dgppo_gnn_attn_*, dgppo_layernorm_*, dgppo_gru_*); torch only
allocates.

Kernel-side parameter layouts (converted from / to the flax layout by `to_flax` / `from_flax`):
  Dense          W (in, out), b (out)                              == flax kernel, bias
  GraphTransformer (D -> F, H heads)
                 Wq (D, H*F), bq (H*F)                             == Dense_0 (query)
                 Wkt (H, F, D), bk (H*F)   Wkt[h] = Dense_1.kernel[:, hF:(h+1)F]^T (key)
                 Wcat (H*(D+5), F) = [Wv (H*D, F); We (H*4, F); bv (H, F)] stacked per head
                   Wv[h*D + d] = Dense_2.kernel[d, hF:(h+1)F], We from Dense_3 (edge, no bias),
                   bv[h] = Dense_2.bias[hF:(h+1)F]
                 Wu (D, F), bu (F)                                 == Dense_4 (update)
  GRUCell(64)    Wi (64, 192) = [ir | iz | in], bi (192), Wh (64, 192) = [hr | hz | hn], bhn (64)
"""
from __future__ import annotations

import math
import os
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from .. import ops
from . import kernels as K

# LayerNorm + ReLU of the MLP heads and the GNN layers' ReLU backward fused into the neighbouring GEMMs' epilogues
# (gemm epi 1-3, ABI 9); DGPPO_FUSE_LN=0 runs the separate layernorm64 / relu_bwd kernels (A/B, parity tests)
FUSE_LN = os.environ.get("DGPPO_FUSE_LN", "1") == "1"
# one GraphTransformer layer forward as ONE kernel ([qt | beta] GEMM + attention + message / update GEMMs, ABI 11
# dgppo_gnn_layer_fwd) where it applies; DGPPO_FUSED_LAYER=0 runs the unfused chain (A/B, parity tests)
FUSED_LAYER = os.environ.get("DGPPO_FUSED_LAYER", "1") == "1"


# ---- parameter space ------------------------------------------------------------------------
class ParamSpace:
    """Flat parameter + gradient buffers with named views.  Every entry starts on a 16-byte boundary
    (the kernels stage weights with 16-byte loads); the padding floats stay zero (zero gradient,
    zero Adam update)."""

    def __init__(self):
        self.entries: List[Tuple[str, Tuple[int, ...], str]] = []
        self.offsets: Dict[str, int] = {}
        self.size = 0
        self.flat = None
        self.grad = None

    def add(self, name: str, shape, init: str) -> str:
        shape = tuple(int(s) for s in shape)
        assert name not in self.offsets, name
        self.offsets[name] = self.size
        self.entries.append((name, shape, init))
        self.size = (self.size + int(np.prod(shape)) + 3) & ~3
        return name

    def build(self, device):
        self.flat = torch.zeros(self.size, dtype=torch.float32, device=device)
        self.grad = torch.zeros(self.size, dtype=torch.float32, device=device)
        return self.build_views()

    def build_views(self):
        self._views = {}
        for n, shape, _ in self.entries:
            o, sz = self.offsets[n], int(np.prod(shape))
            self._views[(n, False)] = self.flat[o:o + sz].view(shape)
            self._views[(n, True)] = self.grad[o:o + sz].view(shape)
        return self

    def view(self, name: str, grad: bool = False) -> torch.Tensor:
        return self._views[(name, bool(grad))]

    def zero_grad(self):
        self.grad.zero_()

    def swap_views(self):
        """Exchange parameter and gradient views (lets the flax exporters export gradients)."""
        for n, _, _ in self.entries:
            self._views[(n, False)], self._views[(n, True)] = self._views[(n, True)], self._views[(n, False)]

    def state_dict(self):
        return {n: self.view(n).detach().cpu().clone() for n, _, _ in self.entries}

    def load_state_dict(self, sd):
        for n, shape, _ in self.entries:
            self.view(n).copy_(torch.as_tensor(sd[n]).reshape(shape))


# ---- host-side initialisers (one-time, not on the hot path) -----------------------------------
def orthogonal(rng: np.random.Generator, shape, scale=1.0):
    """flax.linen.initializers.orthogonal for a (in, out) kernel."""
    n_rows, n_cols = shape
    a = rng.standard_normal((max(n_rows, n_cols), min(n_rows, n_cols)))
    q, r = np.linalg.qr(a)
    q = q * np.sign(np.diag(r))
    if n_rows < n_cols:
        q = q.T
    return (scale * q[:n_rows, :n_cols]).astype(np.float32)


def lecun_normal(rng: np.random.Generator, shape):
    """flax lecun_normal: truncated normal (2 sd) with variance 1 / fan_in."""
    std = math.sqrt(1.0 / shape[0]) / 0.87962566103423978
    x = rng.standard_normal(shape)
    while True:
        bad = np.abs(x) > 2
        if not bad.any():
            break
        x[bad] = rng.standard_normal(bad.sum())
    return (x * std).astype(np.float32)


# ---- building blocks ----------------------------------------------------------------------
class Dense:
    def __init__(self, ps: ParamSpace, name: str, d_in: int, d_out: int, bias=True, init="orthogonal", scale=1.0):
        self.ps, self.name, self.d_in, self.d_out, self.has_bias = ps, name, d_in, d_out, bias
        self.init, self.scale = init, scale
        ps.add(name + ".W", (d_in, d_out), init)
        if bias:
            ps.add(name + ".b", (d_out,), "zeros")

    def W(self, g=False):
        return self.ps.view(self.name + ".W", g)

    def b(self, g=False):
        return self.ps.view(self.name + ".b", g) if self.has_bias else None

    def flax(self) -> dict:
        d = {"kernel": self.W().detach().cpu().numpy()}
        if self.has_bias:
            d["bias"] = self.b().detach().cpu().numpy()
        return d

    def load_flax(self, d):
        self.W().copy_(torch.as_tensor(np.asarray(d["kernel"], np.float32)))
        if self.has_bias:
            self.b().copy_(torch.as_tensor(np.asarray(d["bias"], np.float32)))

    def init_host(self, rng):
        if self.init == "orthogonal":
            w = orthogonal(rng, (self.d_in, self.d_out), self.scale)
        else:
            w = lecun_normal(rng, (self.d_in, self.d_out))
        self.W().copy_(torch.from_numpy(w))

    def fwd(self, x, rows, out=None, relu=False):
        y = out if out is not None else torch.empty((rows, self.d_out), device=x.device)
        K.gemm(x, self.W(), y, rows, self.d_out, self.d_in, bias=self.b(), relu=relu)
        return y

    def bwd(self, x, dy, rows, need_dx=True, dx_out=None, accumulate=False, mask=None, ln=None):
        """dW, db += ...; returns dx.  mask: dx = mask > 0 ? dx : 0 (the input's ReLU backward, fused into the dx
        GEMM); ln: the LayerNorm + ReLU backward of the layer that produced x (GEMM epilogue epi 3)."""
        K.gemm(x, dy, self.W(True), self.d_in, self.d_out, rows, ta=True, beta=1.0, bias_grad=self.b(True))
        if not need_dx:
            return None
        dx = dx_out if dx_out is not None else torch.empty((rows, self.d_in), device=dy.device)
        K.gemm(dy, self.W(), dx, rows, self.d_in, self.d_out, tb=True, ldb=self.d_out, beta=1.0 if accumulate else 0.0,
               mask=mask, ln=ln)
        return dx


class LayerNormReLU:
    def __init__(self, ps: ParamSpace, name: str, F: int):
        self.ps, self.name, self.F = ps, name, F
        ps.add(name + ".scale", (F,), "ones")
        ps.add(name + ".bias", (F,), "zeros")

    def init_host(self, rng):
        self.ps.view(self.name + ".scale").fill_(1.0)

    def flax(self):
        return {"scale": self.ps.view(self.name + ".scale").cpu().numpy(),
                "bias": self.ps.view(self.name + ".bias").cpu().numpy()}

    def load_flax(self, d):
        self.ps.view(self.name + ".scale").copy_(torch.as_tensor(np.asarray(d["scale"], np.float32)))
        self.ps.view(self.name + ".bias").copy_(torch.as_tensor(np.asarray(d["bias"], np.float32)))

    def fwd(self, x):
        rows = x.shape[0]
        y = torch.empty_like(x)
        mean = torch.empty(rows, device=x.device)
        rstd = torch.empty(rows, device=x.device)
        K.layernorm_fwd(x, self.ps.view(self.name + ".scale"), self.ps.view(self.name + ".bias"), y, mean, rstd)
        return y, (x, y, mean, rstd)

    def bwd(self, cache, dy):
        x, y, mean, rstd = cache[:4]
        dx = torch.empty_like(x)
        K.layernorm_bwd(x, y, dy, self.ps.view(self.name + ".scale"), mean, rstd, dx,
                        self.ps.view(self.name + ".scale", True), self.ps.view(self.name + ".bias", True))
        return dx

    # ---- fused into the neighbouring GEMMs (gemm epilogues epi 2 / 3, DGPPO_FUSE_LN=0 keeps the kernels above) ----
    def fwd_fused(self, dense: "Dense", x, rows):
        """y = relu(LayerNorm(x W + b)) as ONE GEMM (its epilogue normalises each 64-wide row); the cache has the
        unfused layout plus a marker, so bwd_args can hand the backward to the next GEMM's epilogue."""
        dev = x.device
        h = torch.empty((rows, self.F), device=dev)
        y = torch.empty((rows, self.F), device=dev)
        mean = torch.empty(rows, device=dev)
        rstd = torch.empty(rows, device=dev)
        K.gemm(x, dense.W(), y, rows, self.F, dense.d_in, bias=dense.b(),
               ln=dict(mode="fwd", scale=self.ps.view(self.name + ".scale"), bias=self.ps.view(self.name + ".bias"),
                       h=h, mean=mean, rstd=rstd))
        return y, (h, y, mean, rstd, "fused")

    def bwd_args(self, cache):
        """The epi 3 argument dict for the GEMM that produces this LayerNorm's output gradient, or None when the
        forward ran unfused (the epilogue reads the fused forward's h, mean and rstd and redoes its ReLU gates bit for bit)."""
        if len(cache) < 5:
            return None
        return dict(mode="bwd", scale=self.ps.view(self.name + ".scale"), bias=self.ps.view(self.name + ".bias"),
                    h=cache[0], mean=cache[2], rstd=cache[3], dscale=self.ps.view(self.name + ".scale", True),
                    dbias=self.ps.view(self.name + ".bias", True))


class MLPHead:
    """MLP(hid_sizes=(64, 64), relu, act_final=True, layernorm) (dgppo/nn/mlp.py:6-30)."""

    def __init__(self, ps, name, d_in=64, hid=64):
        self.d0 = Dense(ps, name + ".Dense_0", d_in, hid)
        self.ln0 = LayerNormReLU(ps, name + ".LayerNorm_0", hid)
        self.d1 = Dense(ps, name + ".Dense_1", hid, hid)
        self.ln1 = LayerNormReLU(ps, name + ".LayerNorm_1", hid)

    def init_host(self, rng):
        for m in (self.d0, self.ln0, self.d1, self.ln1):
            m.init_host(rng)

    def flax(self):
        return {"Dense_0": self.d0.flax(), "LayerNorm_0": self.ln0.flax(), "Dense_1": self.d1.flax(),
                "LayerNorm_1": self.ln1.flax()}

    def load_flax(self, d):
        self.d0.load_flax(d["Dense_0"]), self.ln0.load_flax(d["LayerNorm_0"])
        self.d1.load_flax(d["Dense_1"]), self.ln1.load_flax(d["LayerNorm_1"])

    def fwd(self, x):
        rows = x.shape[0]
        if FUSE_LN and self.d0.d_out == 64 and self.d1.d_out == 64:  # Dense + LayerNorm + ReLU as one GEMM each
            y0, c0 = self.ln0.fwd_fused(self.d0, x, rows)
            y1, c1 = self.ln1.fwd_fused(self.d1, y0, rows)
            return y1, (x, y0, c0, c1)
        h0 = self.d0.fwd(x, rows)
        y0, c0 = self.ln0.fwd(h0)
        h1 = self.d1.fwd(y0, rows)
        y1, c1 = self.ln1.fwd(h1)
        return y1, (x, y0, c0, c1)

    def ln1_bwd_args(self, cache):
        """epi 3 arguments for the GEMM producing d(head output) (the GRU's input-gradient GEMM), or None."""
        return self.ln1.bwd_args(cache[3])

    def bwd(self, cache, dy, need_dx=True, dy_is_dh1=False, mask_input=False):
        """dy = d(head output), or already d(Dense_1 output) when the producer fused LayerNorm_1's backward
        (dy_is_dh1); mask_input: the head input is a ReLU output (the GNN's agent rows), so its ReLU backward is
        fused into the input-gradient GEMM and the caller skips it."""
        x, y0, c0, c1 = cache
        rows = x.shape[0]
        dh1 = dy if dy_is_dh1 else self.ln1.bwd(c1, dy)
        ln0 = self.ln0.bwd_args(c0)
        if ln0 is not None:
            dh0 = self.d1.bwd(y0, dh1, rows, ln=ln0)  # dx GEMM epilogue = LayerNorm_0 + ReLU backward
        else:
            dy0 = self.d1.bwd(y0, dh1, rows)
            dh0 = self.ln0.bwd(c0, dy0)
        return self.d0.bwd(x, dh0, rows, need_dx, mask=x if (mask_input and need_dx) else None)


class GRUCell:
    """flax.linen.GRUCell(features=64) (used through dgppo/nn/rnn.py:15-30)."""

    def __init__(self, ps, name, d_in=64, H=64):
        self.ps, self.name, self.d_in, self.H = ps, name, d_in, H
        ps.add(name + ".Wi", (d_in, 3 * H), "lecun")
        ps.add(name + ".bi", (3 * H,), "zeros")
        ps.add(name + ".Wh", (H, 3 * H), "orthogonal")
        ps.add(name + ".bhn", (H,), "zeros")

    def v(self, k, g=False):
        return self.ps.view(self.name + "." + k, g)

    def init_host(self, rng):
        H = self.H
        wi = np.concatenate([lecun_normal(rng, (self.d_in, H)) for _ in range(3)], axis=1)
        wh = np.concatenate([orthogonal(rng, (H, H)) for _ in range(3)], axis=1)
        self.v("Wi").copy_(torch.from_numpy(wi))
        self.v("Wh").copy_(torch.from_numpy(wh))

    def flax(self):
        H = self.H
        wi, bi, wh, bhn = (self.v(k).cpu().numpy() for k in ("Wi", "bi", "Wh", "bhn"))
        return {"ir": {"kernel": wi[:, :H], "bias": bi[:H]}, "iz": {"kernel": wi[:, H:2 * H], "bias": bi[H:2 * H]},
                "in": {"kernel": wi[:, 2 * H:], "bias": bi[2 * H:]}, "hr": {"kernel": wh[:, :H]},
                "hz": {"kernel": wh[:, H:2 * H]}, "hn": {"kernel": wh[:, 2 * H:], "bias": bhn}}

    def load_flax(self, d):
        wi = np.concatenate([d["ir"]["kernel"], d["iz"]["kernel"], d["in"]["kernel"]], 1).astype(np.float32)
        bi = np.concatenate([d["ir"]["bias"], d["iz"]["bias"], d["in"]["bias"]]).astype(np.float32)
        wh = np.concatenate([d["hr"]["kernel"], d["hz"]["kernel"], d["hn"]["kernel"]], 1).astype(np.float32)
        self.v("Wi").copy_(torch.from_numpy(wi))
        self.v("bi").copy_(torch.from_numpy(bi))
        self.v("Wh").copy_(torch.from_numpy(wh))
        self.v("bhn").copy_(torch.as_tensor(np.asarray(d["hn"]["bias"], np.float32)))

    def seq_fwd(self, x, Q, L, n, h0=None, hs_out=None, hT_out=None):
        """Scan over L steps of Q sequence rows (x rows ordered ((q // n) * L + t) * n + q % n, see
        dgppo_gru_seq_args): one input GEMM + one recurrent kernel.  Returns (hs (Q*L, 64), cache)."""
        rows, H = Q * L, self.H
        gi = torch.empty((rows, 3 * H), device=x.device)
        K.gemm(x, self.v("Wi"), gi, rows, 3 * H, self.d_in, bias=self.v("bi"))
        hs = hs_out if hs_out is not None else torch.empty((rows, H), device=x.device)
        K.gru_seq(True, Q, L, n, gi, self.v("Wh"), self.v("bhn"), h0, hs, hT=hT_out)
        return hs, (x, gi, hs, h0, Q, L, n)

    def seq_bwd(self, cache, dhs, need_dx=True, need_dh0=False, ln=None):
        """Backward of seq_fwd: accumulates dWi, dbi, dWh, dbhn; returns (dx, dh0).  ln: epi 3 arguments of the
        LayerNorm + ReLU that produced x (then dx is the gradient BEFORE that LayerNorm)."""
        x, gi, hs, h0, Q, L, n = cache
        rows, H, dev = Q * L, self.H, dhs.device
        dgi = torch.empty((rows, 3 * H), device=dev)
        dgh = torch.empty((rows, 3 * H), device=dev)
        dh0 = torch.empty((Q, H), device=dev) if need_dh0 else None
        nb = K.gru_seq_blocks(Q)
        part = K.workspace(nb * H, dev, "gru_bhn")
        K.gru_seq(False, Q, L, n, gi, self.v("Wh"), self.v("bhn"), h0, hs, dhs=dhs, dgi=dgi, dgh=dgh, dh0=dh0,
                  dbhn_part=part)
        K.gemm(x, dgi, self.v("Wi", True), self.d_in, 3 * H, rows, ta=True, beta=1.0, bias_grad=self.v("bi", True))
        S = Q // n
        if L > 1:  # h_{t-1} of step t >= 1 is hs of step t-1: row-grouped per sequence, B shifted by n rows
            K.gemm(hs, dgh, self.v("Wh", True), H, 3 * H, S * (L - 1) * n, ta=True, lda=H, a_grp=(L - 1) * n,
                   a_gs=L * n * H, ldb=3 * H, b_off=n * 3 * H, b_grp=(L - 1) * n, b_gs=L * n * 3 * H, beta=1.0)
        if h0 is not None:  # step 0 uses the initial carries
            K.gemm(h0, dgh, self.v("Wh", True), H, 3 * H, Q, ta=True, lda=H, ldb=3 * H, b_grp=n,
                   b_gs=L * n * 3 * H, beta=1.0)
        K.colsum(part, nb, H, self.v("bhn", True), beta=1.0)
        dx = None
        if need_dx:
            dx = torch.empty_like(x)
            K.gemm(dgi, self.v("Wi"), dx, rows, self.d_in, 3 * H, tb=True, ldb=3 * H, ln=ln)
        return dx, dh0

    def fwd(self, x, h, h_out=None):
        """One step for `rows` independent carries (act / get_Vh): (h_new, cache)."""
        rows = h.shape[0]
        return self.seq_fwd(x, rows, 1, 1, h0=h, hs_out=h_out)

    def bwd(self, cache, dhn, need_dx=True):
        """returns (dx, dh)"""
        return self.seq_bwd(cache, dhn, need_dx=need_dx, need_dh0=True)


class LSTMCell:
    """flax.linen.LSTMCell(features=64) (the --use-lstm option of dgppo/nn/rnn.py:21-23): gates
    [i | f | g | o] = x Wi + h Wh + b (the input Denses ii/if/ig/io have no bias, the hidden ones hi/hf/hg/ho
    do), c' = f c + i g, h' = o tanh(c').  Carry rows [c | h] (2 H floats), the reference's stacked (c, h).
    Sequences run time-major inside: one GEMM of every step's input projection, then per step one GEMM of
    the recurrent projection and one gate kernel (dgppo_lstm_cell_fwd / _bwd)."""

    carries = 2

    def __init__(self, ps, name, d_in=64, H=64):
        self.ps, self.name, self.d_in, self.H = ps, name, d_in, H
        ps.add(name + ".Wi", (d_in, 4 * H), "lecun")
        ps.add(name + ".Wh", (H, 4 * H), "orthogonal")
        ps.add(name + ".b", (4 * H,), "zeros")

    def v(self, k, g=False):
        return self.ps.view(self.name + "." + k, g)

    def init_host(self, rng):
        H = self.H
        wi = np.concatenate([lecun_normal(rng, (self.d_in, H)) for _ in range(4)], axis=1)
        wh = np.concatenate([orthogonal(rng, (H, H)) for _ in range(4)], axis=1)
        self.v("Wi").copy_(torch.from_numpy(wi))
        self.v("Wh").copy_(torch.from_numpy(wh))

    _GATES = ("i", "f", "g", "o")

    def flax(self):
        H = self.H
        wi, wh, b = (self.v(k).cpu().numpy() for k in ("Wi", "Wh", "b"))
        d = {}
        for k, gate in enumerate(self._GATES):
            d["i" + gate] = {"kernel": wi[:, k * H:(k + 1) * H]}
            d["h" + gate] = {"kernel": wh[:, k * H:(k + 1) * H], "bias": b[k * H:(k + 1) * H]}
        return d

    def load_flax(self, d):
        f32 = lambda a: np.asarray(a, np.float32)  # noqa: E731
        self.v("Wi").copy_(torch.from_numpy(np.concatenate([f32(d["i" + g]["kernel"]) for g in self._GATES], 1)))
        self.v("Wh").copy_(torch.from_numpy(np.concatenate([f32(d["h" + g]["kernel"]) for g in self._GATES], 1)))
        self.v("b").copy_(torch.from_numpy(np.concatenate([f32(d["h" + g]["bias"]) for g in self._GATES])))

    def seq_fwd(self, x, Q, L, n, h0=None, hs_out=None, hT_out=None):
        """Same contract as GRUCell.seq_fwd, carries (Q, 2H) = [c | h]: returns (hs (Q*L, H), cache)."""
        H, dev = self.H, x.device
        S = Q // n
        xt = x.view(S, L, n, self.d_in).transpose(0, 1).reshape(L * Q, self.d_in)  # rows (t, s, agent)
        G = torch.empty((L, Q, 4 * H), device=dev)
        K.gemm(xt, self.v("Wi"), G.view(L * Q, 4 * H), L * Q, 4 * H, self.d_in)
        cs = torch.empty((L, Q, H), device=dev)
        hst = torch.empty((L, Q, H), device=dev)
        c0 = h0[:, :H].contiguous() if h0 is not None else None
        hh0 = h0[:, H:].contiguous() if h0 is not None else torch.zeros((Q, H), device=dev)
        c_prev, h_prev = c0, hh0
        for t in range(L):
            K.gemm(h_prev, self.v("Wh"), G[t], Q, 4 * H, H, bias=self.v("b"), beta=1.0)
            K.lstm_cell_fwd(Q, H, G[t], c_prev, cs[t], hst[t])
            c_prev, h_prev = cs[t], hst[t]
        hs = hs_out if hs_out is not None else torch.empty((Q * L, H), device=dev)
        hs.view(S, L, n, H).copy_(hst.view(L, S, n, H).transpose(0, 1))
        if hT_out is not None:
            hT_out[:, :H] = cs[L - 1]
            hT_out[:, H:] = hst[L - 1]
        return hs, (xt, G, cs, hst, c0, hh0, Q, L, n)

    def seq_bwd(self, cache, dhs, need_dx=True, need_dh0=False):
        """Backward of seq_fwd: accumulates dWi, dWh, db; returns (dx, dh0 (Q, 2H) = [dc0 | dh0])."""
        xt, G, cs, hst, c0, hh0, Q, L, n = cache
        H, dev = self.H, dhs.device
        S = Q // n
        dht = dhs.view(S, L, n, H).transpose(0, 1).contiguous()  # (L, S, n, H): accumulates the recurrent part
        dht = dht.view(L, Q, H)
        dG = torch.empty((L, Q, 4 * H), device=dev)
        dh0 = torch.empty((Q, 2 * H), device=dev) if need_dh0 else None
        dc = None
        for t in range(L - 1, -1, -1):
            c_prev = cs[t - 1] if t > 0 else c0
            dcp = torch.empty((Q, H), device=dev) if (t > 0 or need_dh0) else None
            K.lstm_cell_bwd(Q, H, G[t], c_prev, cs[t], dht[t], dc, dG[t], dcp)
            if t > 0:
                K.gemm(dG[t], self.v("Wh"), dht[t - 1], Q, H, 4 * H, tb=True, ldb=4 * H, beta=1.0)
            elif need_dh0:
                dh0[:, :H] = dcp
                hpart = torch.empty((Q, H), device=dev)
                K.gemm(dG[0], self.v("Wh"), hpart, Q, H, 4 * H, tb=True, ldb=4 * H)
                dh0[:, H:] = hpart
            dc = dcp
        hprev = torch.cat([hh0.unsqueeze(0), hst[:L - 1]], 0).view(L * Q, H)
        dGf = dG.view(L * Q, 4 * H)
        dWh, db = self.v("Wh", True), self.v("b", True)
        for j in (0, 2 * H):  # two 2H-column halves: the weight-gradient kernel (fused bias colsum) takes N <= 192
            K.gemm(hprev, dGf, dWh, H, 2 * H, L * Q, ta=True, ldb=4 * H, b_off=j, ldc=4 * H, c_off=j, beta=1.0,
                   bias_grad=db[j:j + 2 * H])
        K.gemm(xt, dGf, self.v("Wi", True), self.d_in, 4 * H, L * Q, ta=True, beta=1.0)
        dx = None
        if need_dx:
            dxt = torch.empty((L * Q, self.d_in), device=dev)
            K.gemm(dGf, self.v("Wi"), dxt, L * Q, self.d_in, 4 * H, tb=True, ldb=4 * H)
            dx = dxt.view(L, S, n, self.d_in).transpose(0, 1).reshape(Q * L, self.d_in)
        return dx, dh0


class RNNStack:
    """RNN(rnn_cls, rnn_layers) of dgppo/nn/rnn.py:10-30: `layers` GRUCell / LSTMCell(64) applied in turn (each
    layer's output is the next one's input), or kind "none" (use_rnn=False: the features pass through and the
    carry is kept, policy.py:174-181 / value.py:142-150).  Carry rows hold the reference's (layers, carries, 64)
    flattened: W = layers * carries * 64 floats.  The default (one GRU layer) is exactly GRUCell, same parameter
    names; its carry is the output."""

    def __init__(self, ps, name, kind="gru", layers=1, d_in=64, H=64):
        if kind not in ("gru", "lstm", "none") or layers < 1:
            raise ValueError(f"RNN kind {kind!r}, layers {layers}")
        self.kind, self.H, self.layers = kind, H, layers
        self.carries = 2 if kind == "lstm" else 1
        self.simple = kind == "gru" and layers == 1
        if kind == "none":
            self.cells = []
        elif self.simple:
            self.cells = [GRUCell(ps, name, d_in, H)]
        else:
            cls = GRUCell if kind == "gru" else LSTMCell
            self.cells = [cls(ps, f"{name}.{cls.__name__}_{k}", d_in if k == 0 else H, H) for k in range(layers)]
        self.widths = [getattr(c, "carries", 1) * H for c in self.cells]
        self.W = sum(self.widths) if self.cells else layers * H  # (no RNN: the reference's unused zero carry)

    def init_host(self, rng):
        for c in self.cells:
            c.init_host(rng)

    def flax(self):
        """One GRUCell tree for the default; else the list of cell trees ([] without an RNN)."""
        return self.cells[0].flax() if self.simple else [c.flax() for c in self.cells]

    def load_flax(self, d):
        if self.simple:
            self.cells[0].load_flax(d)
        else:
            for c, dc in zip(self.cells, d):
                c.load_flax(dc)

    def seq_fwd(self, x, Q, L, n, h0=None, hs_out=None, hT_out=None):
        """Scan over L steps of Q carries (GRUCell.seq_fwd's row order); h0 / hT_out (Q, W).  Returns the last
        layer's outputs (Q*L, 64) and the cache."""
        if self.simple:
            return self.cells[0].seq_fwd(x, Q, L, n, h0=h0, hs_out=hs_out, hT_out=hT_out)
        if not self.cells:
            if hT_out is not None:
                if h0 is None:
                    hT_out.zero_()
                else:
                    hT_out.copy_(h0)
            if hs_out is not None:
                hs_out.copy_(x)
                return hs_out, None
            return x, None
        caches, off = [], 0
        for k, (c, w) in enumerate(zip(self.cells, self.widths)):
            h0k = h0[:, off:off + w].contiguous() if h0 is not None else None
            hTk = torch.empty((Q, w), device=x.device) if hT_out is not None else None
            last = k == len(self.cells) - 1
            x, ck = c.seq_fwd(x, Q, L, n, h0=h0k, hT_out=hTk, hs_out=hs_out if last else None)
            if hT_out is not None:
                hT_out[:, off:off + w] = hTk
            caches.append(ck)
            off += w
        return x, caches

    def seq_bwd(self, cache, dhs, need_dx=True, need_dh0=False, ln=None):
        """Backward of seq_fwd: returns (dx, dh0 (Q, W)).  ln (the 1-layer GRU only; see fuses_ln): the input's
        LayerNorm + ReLU backward fused into the input-gradient GEMM."""
        if self.simple:
            return self.cells[0].seq_bwd(cache, dhs, need_dx=need_dx, need_dh0=need_dh0, ln=ln)
        assert ln is None, "LayerNorm-fused input gradient: 1-layer GRU only"
        if not self.cells:
            return (dhs if need_dx else None), (torch.zeros((dhs.shape[0], self.W), device=dhs.device)
                                                if need_dh0 else None)
        dh0s = []
        d = dhs
        for k in range(len(self.cells) - 1, -1, -1):
            d, dh0k = self.cells[k].seq_bwd(cache[k], d, need_dx=need_dx or k > 0, need_dh0=need_dh0)
            dh0s.append(dh0k)
        dh0 = torch.cat(dh0s[::-1], 1) if need_dh0 else None
        return d, dh0

    def fwd(self, x, h, h_out=None):
        """One step for `rows` independent carries h (rows, W) (act / get_Vh): (output (rows, 64), new carries
        (rows, W), cache)."""
        rows = h.shape[0]
        if self.simple:
            h2, c = self.cells[0].fwd(x, h, h_out=h_out)
            return h2, h2, c
        h2 = h_out if h_out is not None else torch.empty((rows, self.W), device=h.device)
        y, c = self.seq_fwd(x, rows, 1, 1, h0=h, hT_out=h2)
        return y, h2, c

    def bwd(self, cache, dy, need_dx=True, ln=None):
        """returns (dx, dh)"""
        return self.seq_bwd(cache, dy, need_dx=need_dx, need_dh0=True, ln=ln)


class GraphTransformer:
    """GraphTransformer layer (dgppo/nn/gnn.py:78-117) in the per-receiving-agent form."""

    def __init__(self, ps, name, D, F, H=3, ED=4):
        self.ps, self.name, self.D, self.F, self.H = ps, name, D, F, H
        self.ED, self.EX = ED, ED - 4  # edge width; columns past the first 4 go through Wex
        if ED < 4:
            raise ValueError(f"edge_dim {ED} < 4")
        ps.add(name + ".Wq", (D, H * F), "orthogonal")
        ps.add(name + ".bq", (H * F,), "zeros")
        ps.add(name + ".Wkt", (H, F, D), "orthogonal")
        ps.add(name + ".bk", (H * F,), "zeros")
        ps.add(name + ".Wcat", (H * (D + 5), F), "orthogonal")
        ps.add(name + ".Wu", (D, F), "orthogonal")
        ps.add(name + ".bu", (F,), "zeros")
        if self.EX:
            ps.add(name + ".Wex", (H * self.EX, F), "orthogonal")  # Dense_3 rows 4.. as (head, column, F)

    def v(self, k, g=False):
        return self.ps.view(self.name + "." + k, g)

    # ---- flax layout conversion (Dense_0..Dense_4 of the reference) ----
    def load_flax(self, d):
        D, F, H = self.D, self.F, self.H
        f32 = lambda a: np.asarray(a, np.float32)  # noqa: E731
        self.v("Wq").copy_(torch.from_numpy(f32(d["Dense_0"]["kernel"])))
        self.v("bq").copy_(torch.from_numpy(f32(d["Dense_0"]["bias"])))
        wk = f32(d["Dense_1"]["kernel"]).reshape(D, H, F).transpose(1, 2, 0)  # (H, F, D)
        self.v("Wkt").copy_(torch.from_numpy(np.ascontiguousarray(wk)))
        self.v("bk").copy_(torch.from_numpy(f32(d["Dense_1"]["bias"])))
        wv = f32(d["Dense_2"]["kernel"]).reshape(D, H, F).transpose(1, 0, 2).reshape(H * D, F)
        k3 = f32(d["Dense_3"]["kernel"]).reshape(self.ED, H, F)
        we = k3[:4].transpose(1, 0, 2).reshape(H * 4, F)
        if self.EX:
            self.v("Wex").copy_(torch.from_numpy(np.ascontiguousarray(k3[4:].transpose(1, 0, 2).reshape(H * self.EX, F))))
        bv = f32(d["Dense_2"]["bias"]).reshape(H, F)
        self.v("Wcat").copy_(torch.from_numpy(np.concatenate([wv, we, bv], 0)))
        self.v("Wu").copy_(torch.from_numpy(f32(d["Dense_4"]["kernel"])))
        self.v("bu").copy_(torch.from_numpy(f32(d["Dense_4"]["bias"])))

    def flax(self):
        D, F, H = self.D, self.F, self.H
        wcat = self.v("Wcat").cpu().numpy()
        wv, we, bv = wcat[:H * D], wcat[H * D:H * D + 4 * H], wcat[H * D + 4 * H:]
        k3 = we.reshape(H, 4, F).transpose(1, 0, 2).reshape(4, H * F)
        if self.EX:
            wex = self.v("Wex").cpu().numpy().reshape(H, self.EX, F).transpose(1, 0, 2).reshape(self.EX, H * F)
            k3 = np.concatenate([k3, wex], 0)
        return {
            "Dense_0": {"kernel": self.v("Wq").cpu().numpy(), "bias": self.v("bq").cpu().numpy()},
            "Dense_1": {"kernel": self.v("Wkt").cpu().numpy().transpose(2, 0, 1).reshape(D, H * F),
                        "bias": self.v("bk").cpu().numpy()},
            "Dense_2": {"kernel": wv.reshape(H, D, F).transpose(1, 0, 2).reshape(D, H * F), "bias": bv.reshape(-1)},
            "Dense_3": {"kernel": k3},
            "Dense_4": {"kernel": self.v("Wu").cpu().numpy(), "bias": self.v("bu").cpu().numpy()},
        }

    def init_host(self, rng):
        D, F, H = self.D, self.F, self.H
        d = {"Dense_0": {"kernel": orthogonal(rng, (D, H * F)), "bias": np.zeros(H * F, np.float32)},
             "Dense_1": {"kernel": orthogonal(rng, (D, H * F)), "bias": np.zeros(H * F, np.float32)},
             "Dense_2": {"kernel": orthogonal(rng, (D, H * F)), "bias": np.zeros(H * F, np.float32)},
             "Dense_3": {"kernel": orthogonal(rng, (self.ED, H * F))},
             "Dense_4": {"kernel": orthogonal(rng, (D, F)), "bias": np.zeros(F, np.float32)}}
        self.load_flax(d)

    def _attn_args(self, g: "GraphBatch", QB, xa=None, pre=None, xfull=None) -> dict:
        """Inputs of torch.ops.dgppo.gnn_attn_fwd / _bwd for this layer on graph batch g, Q-free form:
        QB (R, H*D + H) = [qt | beta] rows (see qb_weights).  xfull (G, N, D): every node's input row
        (layers past the second of a deeper GNN), else the raw nodes (first layer) or agent mode."""
        D0 = 0
        pre_W = pre_b = None
        if xfull is not None:
            x, x_gs = xfull, g.N * self.D
        elif xa is None:
            x, x_gs = g.nodes, g.N * g.nodes.shape[2]
        else:  # agent mode: agents from xa, other senders = pre's Dense_4 + ReLU of raw rows
            raw, cols = g.sender_raw
            D0 = raw.shape[2]
            x, x_gs = raw, g.N * D0
            if pre is not None:
                pre_W = pre.v("Wu") if cols is None else pre.v("Wu").index_select(0, cols)
                pre_b = pre.v("bu")
        HD = self.H * self.D
        W = HD + self.H
        return dict(dims=[g.G, g.N, g.E, g.n, self.D, self.F, self.H, g.C, D0], cand=g.cand, receivers=g.receivers,
                    senders=g.senders, sidx=g.sidx, x=x, x_gstride=x_gs, ef=g.edges_head, ef_gstride=g.E * 4, q=None,
                    qt=QB, bk=self.v("bk"), scale=1.0 / math.sqrt(self.F), xa=xa, xa_gstride=g.n * self.D,
                    pre_W=pre_W, pre_b=pre_b, beta=QB[:, HD:], beta_ld=W, qt_ld=W)

    def _aug(self, w: str, b: str, grad=False) -> torch.Tensor:
        """[W; b] as one ((in+1), out) view: the flat buffer stores a Dense's kernel then its bias."""
        ow, ob = self.ps.offsets[self.name + "." + w], self.ps.offsets[self.name + "." + b]
        rows, cols = self.ps.view(self.name + "." + w).shape
        assert ob == ow + rows * cols, "bias must follow its kernel in the flat buffer"
        buf = self.ps.grad if grad else self.ps.flat
        return buf[ow:ow + (rows + 1) * cols].view(rows + 1, cols)

    def qb_weights(self) -> torch.Tensor:
        """QBW ((D+1), H*D + H): with q_h = x Wq_h + bq_h, the attention needs only qt_h = q_h Wkt_h (its
        logits are (qt_h . x_s + q_h . bk_h) / sqrt(F)) and beta_h = q_h . bk_h, both affine in x:
        [x 1] QBW = [qt | beta] with QBW[:, hD:(h+1)D] = [Wq_h; bq_h] Wkt_h and QBW[:, HD + h] =
        [Wq_h; bq_h] bk_h.  Two small batched GEMMs on the weights replace materialising q (R, H*F)."""
        D, F, H = self.D, self.F, self.H
        W = H * D + H
        Waug = self._aug("Wq", "bq")
        QBW = torch.empty((D + 1, W), device=Waug.device)
        K.gemm(Waug, self.v("Wkt"), QBW, D + 1, D, F, lda=H * F, sa=F, ldb=D, sb=F * D, ldc=W, sc=D, batch=H)
        K.gemm(Waug, self.v("bk"), QBW, D + 1, 1, F, lda=H * F, sa=F, ldb=1, sb=F, ldc=W, sc=1, c_off=H * D, batch=H)
        return QBW

    def _fused_fwd(self, g: "GraphBatch", xa, pre, keep: bool, zmean=None, tail=None):
        """The layer through dgppo_gnn_layer_fwd (one kernel), or None where it does not apply.  keep: also write
        [qt | beta], attn and xcat for the backward (else Y only, forward-only passes).  Forward-only epilogues (keep
        False): zmean (G, F) receives the per-graph agent mean of Y, and Y is not written; tail = (weights in
        ops.TAIL_FIELDS order, carries (G*n, 64), out (G*n, n_out)) runs the value head after the layer (the return
        value is then (out, None))."""
        if (xa is not None and pre is None) or self.EX:
            return None
        G, n, D, F, H, C = g.G, g.n, self.D, self.F, self.H, g.C
        R, W = G * n, H * D + H
        dev = g.nodes.device
        if xa is None:
            x, x_gs, D0, pre_W, pre_b = g.nodes, g.N * g.nodes.shape[2], 0, None, None
        else:
            raw, cols = g.sender_raw
            if cols is not None:
                return None
            x, x_gs, D0, pre_W, pre_b = raw, g.N * raw.shape[2], raw.shape[2], pre.v("Wu"), pre.v("bu")
        QBW = self.qb_weights()
        Y = torch.empty((R, F), device=dev) if (zmean is None and tail is None) else None
        tail_w, tail_h, tail_out = tail if tail is not None else ([], None, None)
        kw = dict(dims=[G, g.N, g.E, n, D, F, H, C, D0], cand=g.cand, receivers=g.receivers, senders=g.senders,
                  sidx=g.sidx, x=x, x_gstride=x_gs, ef=g.edges_head, ef_gstride=g.E * 4, scale=1.0 / math.sqrt(F),
                  xa=xa, xa_gstride=n * D, pre_W=pre_W, pre_b=pre_b, QBW=QBW, Wcat=self.v("Wcat"), Wu=self.v("Wu"),
                  bu=self.v("bu"), Y=Y, zmean=zmean, tail_w=tail_w, tail_h=tail_h, tail_out=tail_out)
        if not ops.gnn_layer_supported(**kw):
            return None
        QB = attn = xcat = None
        if keep:
            QB = torch.empty((R, W), device=dev)
            attn = torch.empty((R, H, C), device=dev)
            xcat = torch.empty((R, H * (D + 5)), device=dev)
        o = kw
        torch.ops.dgppo.gnn_layer_fwd(o["dims"], o["cand"], o["receivers"], o["senders"], o["sidx"], o["x"],
                                      o["x_gstride"], o["ef"], o["ef_gstride"], o["scale"], o["xa"], o["xa_gstride"],
                                      o["pre_W"], o["pre_b"], o["QBW"], o["Wcat"], o["Wu"], o["bu"], Y, QB, attn, xcat,
                                      zmean, list(tail_w), tail_h, tail_out)
        if tail is not None:
            return tail_out, None
        if zmean is not None:
            return zmean, None
        return Y, ((xa, pre, QBW, QB, attn, xcat, None, Y, None) if keep else None)

    def fwd(self, g: "GraphBatch", xa=None, pre=None, xfull=None, keep=True):
        """One layer on the graph batch.  xa None: senders read the raw nodes (G, N, D) (first layer);
        else xa (G*n, D) holds the agents' rows and the never-receiving nodes are `pre`'s
        Dense_4 + ReLU of their raw rows (agent mode); xfull (G, N, D): every node's row given
        (GNN layers past the second).  Returns Y (G*n, F) = the agents' outputs (only agents
        receive, so only their rows feed the next layer's queries) and the cache.
        Edge columns past the first 4 add (sum_c attn * efx) @ Wex to the messages (edge_wsum).
        keep=False: forward only (the fused kernel then skips the backward's intermediates; cache None)."""
        self.last_fused = False  # which path the last call took (tests)
        if FUSED_LAYER and xfull is None and not self.EX:
            out = self._fused_fwd(g, xa, pre, keep)
            if out is not None:
                self.last_fused = True
                return out
        G, N, n = g.G, g.N, g.n
        D, F, H, C = self.D, self.F, self.H, g.C
        dev = g.nodes.device
        R = G * n
        A, akw = self._rows_in(g, xa, xfull)
        QBW = self.qb_weights()
        W = H * D + H
        QB = torch.empty((R, W), device=dev)  # [qt | beta] per receiving agent: one GEMM, q never stored
        K.gemm(A, QBW, QB, R, W, D, bias=QBW[D], **akw)
        attn = torch.empty((R, H, C), device=dev)
        xcat = torch.empty((R, H * (D + 5)), device=dev)
        torch.ops.dgppo.gnn_attn_fwd(**self._attn_args(g, QB, xa, pre, xfull), attn=attn, xcat=xcat)
        M = torch.empty((R, F), device=dev)
        K.gemm(xcat, self.v("Wcat"), M, R, F, H * (D + 5), alpha=1.0 / H)
        xcx = None
        if self.EX:
            xcx = torch.empty((R, H * self.EX), device=dev)
            K.edge_wsum(G, n, C, H, self.EX, g.E, attn, g.cand, g.sidx, g.edges_x, xcx)
            K.gemm(xcx, self.v("Wex"), M, R, F, H * self.EX, alpha=1.0 / H, beta=1.0)
        Y = torch.empty((R, F), device=dev)
        K.gemm(A, self.v("Wu"), Y, R, F, D, bias=self.v("bu"), addend=M, relu=True, **akw)
        return Y, ((xa, pre, QBW, QB, attn, xcat, xcx, Y, xfull) if keep else None)

    def _rows_in(self, g: "GraphBatch", xa, xfull):
        """The receiving agents' input rows as a GEMM operand: (tensor, row-grouping kwargs)."""
        if xa is not None:
            return xa, dict(lda=self.D)
        x = xfull if xfull is not None else g.nodes
        return x, dict(lda=self.D, a_grp=g.n, a_gs=g.N * self.D)

    def _pre_grads(self, pre, g, part, nb, PK, D0):
        """Sum the per-workgroup [Wu (D0 x D) | bu (D)] partial rows of the pre layer (Wu rows = the raw columns used)."""
        D, dev = self.D, part.device
        cols = g.sender_raw[1]
        ow, ob = pre.ps.offsets[pre.name + ".Wu"], pre.ps.offsets[pre.name + ".bu"]
        nw = D0 * D
        if ob == ow + nw and cols is None:
            K.colsum(part, nb, PK, pre.ps.grad[ow:ow + PK], beta=1.0)
        else:
            tmp = torch.empty(PK, device=dev)
            K.colsum(part, nb, PK, tmp)
            if cols is None:
                pre.ps.grad[ow:ow + nw].add_(tmp[:nw])
            else:
                pre.v("Wu", True).index_add_(0, cols, tmp[:nw].view(D0, D))
            pre.ps.grad[ob:ob + D].add_(tmp[nw:])

    def _qfree_grads(self, A, akw, dQB, R):
        """Q-free parameter gradients: Gaug = [x 1]^T [dqt | dbeta] ((D+1) x (HD+H)), one pass over the rows; then,
        per head, with Waug_h = [Wq_h; bq_h] ((D+1) x F):
          [dWq_h; dbq_h] += Gaug[:, hD:(h+1)D] Wkt_h^T + Gaug[:, HD+h] bk_h^T
          dWkt_h += Waug_h^T Gaug[:, hD:(h+1)D],   dbk_h += Waug_h^T Gaug[:, HD+h]
        (q_h = x Wq_h + bq_h is affine in the layer input, so every sum over rows of q collapses into Gaug)"""
        D, F, H = self.D, self.F, self.H
        HD, WQ = H * D, H * D + H
        Gaug = torch.empty((D + 1, WQ), device=dQB.device)
        K.gemm(A, dQB, Gaug, D, WQ, R, ta=True, bias_grad=Gaug[D], **akw)
        Waug, dWaug = self._aug("Wq", "bq"), self._aug("Wq", "bq", grad=True)
        K.gemm(Gaug, self.v("Wkt"), dWaug, D + 1, F, D, lda=WQ, sa=D, tb=True, ldb=D, sb=F * D, ldc=H * F, sc=F,
               batch=H, beta=1.0)
        K.gemm(Gaug, self.v("bk"), dWaug, D + 1, F, 1, lda=WQ, a_off=HD, sa=1, ldb=F, sb=F, ldc=H * F, sc=F,
               batch=H, beta=1.0)
        K.gemm(Waug, Gaug, self.v("Wkt", True), F, D, D + 1, ta=True, lda=H * F, sa=F, ldb=WQ, sb=D, ldc=D,
               sc=F * D, batch=H, beta=1.0)
        K.gemm(Waug, Gaug, self.v("bk", True), F, 1, D + 1, ta=True, lda=H * F, sa=F, ldb=WQ, b_off=HD, sb=1,
               ldc=1, sc=F, batch=H, beta=1.0)

    def bwd(self, cache, dY, g: "GraphBatch", masked=False, mask_dxa=False):
        """dY (G*n, F) is consumed (becomes dZ).  Returns d xa (G*n, D) in agent mode, d xfull (G, N, D)
        when every node's row was given, else None; accumulates this layer's grads and, in agent mode
        with `pre`, pre's Dense_4 grads from the transformed senders.  masked: dY already carries this layer's
        ReLU gate (its producer's GEMM epilogue applied it); mask_dxa: apply the previous layer's ReLU gate
        (xa > 0) in the last GEMM that forms d xa, so the previous layer's bwd runs with masked=True."""
        xa, pre, QBW, QB, attn, xcat, xcx, Y, xfull = cache
        G, N, n = g.G, g.N, g.n
        D, F, H, C = self.D, self.F, self.H, g.C
        R = G * n
        W = H * (D + 5)
        HD, WQ = H * D, H * D + H
        dev = dY.device
        A, akw = self._rows_in(g, xa, xfull)
        if not masked:
            K.relu_bwd_(dY, Y)  # dY := dZ
        dxcat = torch.empty((R, W), device=dev)
        K.gemm(dY, self.v("Wcat"), dxcat, R, W, F, tb=True, ldb=F, alpha=1.0 / H)
        K.gemm(xcat, dY, self.v("Wcat", True), W, F, R, ta=True, lda=W, alpha=1.0 / H, beta=1.0)
        da_add = None
        if self.EX:
            WX = H * self.EX
            dxx = torch.empty((R, WX), device=dev)
            K.gemm(dY, self.v("Wex"), dxx, R, WX, F, tb=True, ldb=F, alpha=1.0 / H)
            K.gemm(xcx, dY, self.v("Wex", True), WX, F, R, ta=True, lda=WX, alpha=1.0 / H, beta=1.0)
            da_add = torch.empty((R, H, C), device=dev)
            K.edge_da(G, n, C, H, self.EX, g.E, dxx, g.cand, g.sidx, g.edges_x, da_add)
        dQB = torch.empty((R, WQ), device=dev)  # [dqt | dbeta]
        dXa = torch.zeros((R, D), device=dev) if xa is not None else None
        dXf = torch.zeros((G, N, D), device=dev) if xfull is not None else None  # every sender's gradient
        args = self._attn_args(g, QB, xa, pre, xfull)
        part = None
        if xa is not None and pre is not None:
            nb = ops.gnn_attn_partial_blocks(**args)
            PK = args["dims"][8] * D + D
            part = K.workspace(nb * PK, dev, "attn_pre")
        torch.ops.dgppo.gnn_attn_bwd(**args, attn=attn, dxcat=dxcat, da_add=da_add, dqt=dQB, dq=None,
                                     dbeta=dQB[:, HD:], dxa=dXa, dxa_gstride=n * D, dpre_part=part, dqt_ld=WQ,
                                     dbeta_ld=WQ, dx=dXf, dx_gstride=N * D)
        if part is not None:
            self._pre_grads(pre, g, part, nb, PK, args["dims"][8])
        self._qfree_grads(A, akw, dQB, R)  # parameter gradients only
        K.gemm(A, dY, self.v("Wu", True), D, F, R, ta=True, beta=1.0, bias_grad=self.v("bu", True), **akw)
        if dXa is not None:
            K.gemm(dY, self.v("Wu"), dXa, R, D, F, tb=True, ldb=F, beta=1.0)
            K.gemm(dQB, QBW, dXa, R, D, WQ, tb=True, ldb=WQ, beta=1.0,  # d[qt | beta] / dx = QBW[:D]^T
                   mask=xa if mask_dxa else None)
            return dXa
        if dXf is not None:  # the agents' rows also fed Dense_4 and the queries: added in place (row-grouped C)
            cg = dict(c_grp=n, c_gs=N * D, ldc=D, beta=1.0)
            K.gemm(dY, self.v("Wu"), dXf, R, D, F, tb=True, ldb=F, **cg)
            K.gemm(dQB, QBW, dXf, R, D, WQ, tb=True, ldb=WQ, **cg)
            return dXf
        return None


_COLS = {}


class GraphBatch:
    """A batch of env graphs as the GNN kernels consume them (nodes/edges/receivers/senders contiguous
    (G, ...)), plus the per-agent candidate-edge table of the env layout.

    raw_cols: the node-feature columns a never-receiving node (goal, obstacle, lidar hit) can have nonzero
    (env.nonagent_feature_cols); needed when the node width exceeds the attention kernels' raw-row limit
    (8), e.g. LidarOmniTarget's 10-wide nodes: agent-mode layers then read those columns only."""

    KD0 = 8  # attn.hip kD0

    @staticmethod
    def from_graph(graph, env, flatten_dims=None):
        """GraphsTuple with any leading batch dims -> GraphBatch over all graphs (row-major)."""
        nd = graph.nodes.dim() - 2
        G = int(np.prod(graph.nodes.shape[:nd]))
        return GraphBatch(graph.nodes.reshape(G, *graph.nodes.shape[nd:]), graph.edges.reshape(G, *graph.edges.shape[nd:]),
                          graph.receivers.reshape(G, -1), graph.senders.reshape(G, -1), env.num_agents,
                          env.agent_candidates(graph.nodes.device), raw_cols=getattr(env, "nonagent_feature_cols", None))

    def __init__(self, nodes, edges, receivers, senders, n_agents: int, cand: torch.Tensor, raw_cols=None):
        self.nodes = nodes.contiguous()
        self.edges = edges.contiguous()
        self.receivers = receivers.contiguous()
        self.senders = senders.contiguous()
        self.G, self.N = self.nodes.shape[0], self.nodes.shape[1]
        self.E = self.edges.shape[1]
        self.ED = self.edges.shape[2]
        self.n = int(n_agents)
        self.cand = cand
        self.C = int(cand.shape[1])
        self.raw_cols = tuple(int(c) for c in raw_cols) if raw_cols is not None else None
        self._sidx = None
        self._edges_head = self._edges_x = self._sender_raw = None

    def prepare(self):
        """Build every lazily derived table (sender table, edge splits, raw sender rows) now, on the
        current stream, so the batch can be read by passes running concurrently on other streams."""
        _ = self.sidx, self.edges_head, self.edges_x, self.sender_raw
        return self

    @property
    def sidx(self) -> torch.Tensor:
        """(G*n, C) resolved sender of every candidate edge (-1 if masked), built once per batch and
        shared by every attention launch on it."""
        if self._sidx is None:
            self._sidx = torch.empty((self.G * self.n, self.C), dtype=torch.int32, device=self.nodes.device)
            K.sender_table(self.G, self.n, self.C, self.E, self.cand, self.receivers, self.senders, self._sidx)
        return self._sidx

    @property
    def edges_head(self) -> torch.Tensor:
        """(G, E, 4): the edge columns the attention kernels read."""
        if self.ED == 4:
            return self.edges
        if self._edges_head is None:
            self._edges_head = self.edges[..., :4].contiguous()
        return self._edges_head

    @property
    def edges_x(self):
        """(G, E, ED-4) the remaining edge columns (None for 4-wide edges)."""
        if self.ED == 4:
            return None
        if self._edges_x is None:
            self._edges_x = self.edges[..., 4:].contiguous()
        return self._edges_x

    @property
    def sender_raw(self):
        """(raw rows the agent-mode layers read for never-receiving senders, column index tensor or None)."""
        if self._sender_raw is None:
            D0 = self.nodes.shape[2]
            if D0 <= self.KD0:
                self._sender_raw = (self.nodes, None)
            else:
                if self.raw_cols is None or len(self.raw_cols) > self.KD0:
                    raise NotImplementedError(
                        f"node width {D0} > {self.KD0} needs raw_cols (<= {self.KD0} columns) for agent-mode layers")
                key = (self.raw_cols, str(self.nodes.device))
                if key not in _COLS:  # created once per device, so hipGraph capture never sees the H2D copy
                    _COLS[key] = torch.tensor(self.raw_cols, dtype=torch.int64, device=self.nodes.device)
                cols = _COLS[key]
                self._sender_raw = (self.nodes.index_select(2, cols).contiguous(), cols)
        return self._sender_raw


class GNN:
    """GraphTransformerGNN (dgppo/nn/gnn.py:127-142), msg_dim 32, out_dim 64, 3 heads, followed by
    type_nodes(agent): returns the agent rows of the last layer, (G*n, out_dim)."""

    def __init__(self, ps, name, node_dim, n_layers, msg_dim=32, out_dim=64, n_heads=3, edge_dim=4):
        if n_layers < 1:
            raise ValueError(f"GNN depth {n_layers} < 1")
        self.layers = []
        d = node_dim
        for i in range(n_layers):
            od = out_dim if i == n_layers - 1 else msg_dim
            self.layers.append(GraphTransformer(ps, f"{name}.GraphTransformer_{i}", d, od, n_heads, edge_dim))
            d = od

    def init_host(self, rng):
        for L in self.layers:
            L.init_host(rng)

    def flax(self):
        return [L.flax() for L in self.layers]

    def load_flax(self, layers):
        for L, d in zip(self.layers, layers):
            L.load_flax(d)

    def _lift(self, Z, i, rows):
        """Z_{i+1} = relu(Z_i Wu_i + bu_i) over every node row: the layer-(i+1) input of a node that never
        receives (goals, hits, obstacles: empty aggregation, gnn.py:110-117)."""
        L = self.layers[i]
        out = torch.empty((rows, L.F), device=Z.device)
        K.gemm(Z, L.v("Wu"), out, rows, L.F, L.D, bias=L.v("bu"), relu=True)
        return out

    def fwd_epilogue(self, g: GraphBatch, zmean=None, tail=None):
        """Forward only, with the last layer's fused epilogue (GraphTransformer._fused_fwd: zmean = the agent mean of
        its output, tail = the value head): the epilogue's output, or None where the fused kernels do not cover the
        stack (the caller then runs fwd() and the unfused head)."""
        # 10-wide edges (EX > 0) need the edge_wsum term the fused kernel does not add: decline before launching
        if not FUSED_LAYER or len(self.layers) > 2 or any(L.EX for L in self.layers):
            return None
        Y = None
        for i, L in enumerate(self.layers):
            last = i == len(self.layers) - 1
            kw = dict(zmean=zmean, tail=tail) if last else {}
            out = L._fused_fwd(g, Y if i else None, self.layers[0] if i else None, False, **kw)
            if out is None:
                return None
            Y = out[0]
        return Y

    def fwd(self, g: GraphBatch, keep=True):
        """Layer 0 reads the raw nodes, layer 1 runs in agent mode (never-receivers' layer-1 rows recomputed
        from the raw rows in the kernel).  Layers l >= 2 (deeper stacks than the reference's defaults) read
        materialised rows X_l (G, N, D): the agents' rows are the previous layer's outputs, every other
        node's row is Z_l = relu(Z_{l-1} Wu_{l-1} + bu_{l-1}) from Z_0 = the raw nodes."""
        caches = []
        Y = None
        G, N, n = g.G, g.N, g.n
        Zs = [g.nodes.reshape(G * N, g.nodes.shape[2])] if len(self.layers) > 2 else None
        for i, L in enumerate(self.layers):
            if i == 0:
                Y, c = L.fwd(g, keep=keep)
            elif i == 1:
                Y, c = L.fwd(g, xa=Y, pre=self.layers[0], keep=keep)
            else:
                while len(Zs) <= i:
                    Zs.append(self._lift(Zs[-1], len(Zs) - 1, G * N))
                X = Zs[i].view(G, N, L.D).clone()
                X[:, :n] = Y.view(G, n, L.D)
                Y, c = L.fwd(g, xfull=X, keep=keep)
            caches.append(c)
        return Y, ((caches, Zs) if keep else None)

    def bwd(self, caches, dZ, g: GraphBatch, top_masked=False):
        """top_masked: dZ already carries the last layer's ReLU gate (fused into its producer's GEMM)."""
        caches, Zs = caches
        G, N, n = g.G, g.N, g.n
        rows = G * N
        d = dZ
        fused_in = False
        acc = None  # gradient of the never-receivers' lifted rows Z_i (rows, D_i), deep stacks only
        for i in range(len(self.layers) - 1, -1, -1):
            L = self.layers[i]
            if i >= 2:
                dX = L.bwd(caches[i], d, g)  # (G, N, D_i): every sender's row
                d = dX[:, :n].reshape(G * n, L.D).contiguous()
                dX[:, :n] = 0.0  # agents' rows came from the previous layer, not from the lift
                dz = dX.view(rows, L.D)
                if acc is not None:
                    dz.add_(acc)
                P = self.layers[i - 1]  # Z_i = relu(Z_{i-1} Wu_{i-1} + bu_{i-1})
                K.relu_bwd_(dz, Zs[i])
                K.gemm(Zs[i - 1], dz, P.v("Wu", True), P.D, P.F, rows, ta=True, beta=1.0, bias_grad=P.v("bu", True))
                acc = None
                if i - 1 >= 1:
                    acc = torch.empty((rows, P.D), device=dz.device)
                    K.gemm(dz, P.v("Wu"), acc, rows, P.D, P.F, tb=True, ldb=P.F)
                continue
            if i == 1 and acc is not None:  # Z_1 = relu(Z_0 Wu_0 + bu_0) of the raw rows Z_0
                P = self.layers[0]
                K.relu_bwd_(acc, Zs[1])
                K.gemm(Zs[0], acc, P.v("Wu", True), P.D, P.F, rows, ta=True, beta=1.0, bias_grad=P.v("bu", True))
                acc = None
            last = i == len(self.layers) - 1
            d = L.bwd(caches[i], d, g, masked=(top_masked if last else fused_in), mask_dxa=(i == 1 and FUSE_LN))
            fused_in = i == 1 and FUSE_LN  # layer 0's dY got its ReLU gate in layer 1's d xa GEMM

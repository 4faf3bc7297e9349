"""float64 torch-CPU twin of oracle/nets.py used for GRADIENT checks (autograd on the reference's
literal per-edge formulation).  TEST INFRASTRUCTURE ONLY; see oracle/__init__.py.

Same param trees as oracle/nets.py (flax layout); every leaf is a float64 tensor that may require
grad.  Function-for-function restatement of dgppo/nn/gnn.py:78-142, dgppo/nn/mlp.py:15-30,
flax GRUCell, dgppo/algo/module/policy.py:61-74, value.py:15-79, distribution.py:10-66,
informarl.py:357-457 and dgppo.py:296-321."""
from __future__ import annotations

import math

import numpy as np
import torch

T64 = torch.float64


def to_t(tree, requires_grad=False):
    if isinstance(tree, dict):
        return {k: to_t(v, requires_grad) for k, v in tree.items()}
    if isinstance(tree, (list, tuple)):
        return [to_t(v, requires_grad) for v in tree]
    t = torch.tensor(np.asarray(tree), dtype=T64)
    if requires_grad:
        t.requires_grad_(True)
    return t


def dense(x, p):
    y = x @ p["kernel"]
    return y + p["bias"] if "bias" in p else y


# Test instrument for ReLU gates that fp32 rounding decides (tests/test_update_dynamics_gpu.py): with GATE_MODE
# "on" / "off", a GNN update ReLU whose float64 pre-activation lies within GATE_TAU of the fp32 rounding scale of
# its dot product (|x| |W| + |b|) of zero, or an MLP-head ReLU(LayerNorm) output within GATE_TAU_LN of zero, is
# forced open / shut (value 0 or the pre-activation itself, gradient 1 or 0); None keeps torch.relu.  Any fp32
# implementation may take either decision for such an entry.
GATE_MODE = None
GATE_TAU = 8 * 2.0 ** -24
GATE_TAU_LN = 1e-5
# when a list: every gated call under GATE_MODE "on" appends (ambiguous gates, gates evaluated), so the test can
# bound how many decisions the fallback tolerance covers
GATE_STATS = None


def _gate_count(amb):
    if GATE_STATS is not None and GATE_MODE == "on":
        GATE_STATS.append((int(amb.sum().item()), int(amb.numel())))


def _gnn_relu(pre, x, p):
    if GATE_MODE is None:
        return torch.relu(pre)
    with torch.no_grad():
        scale = x.abs() @ p["kernel"].abs() + (p["bias"].abs() if "bias" in p else 0.0)
        amb = pre.abs() <= GATE_TAU * scale
        _gate_count(amb)
    forced = pre if GATE_MODE == "on" else pre * 0.0
    return torch.where(amb, forced, torch.relu(pre))


def layernorm(x, p, eps=1e-6):
    mean = x.mean(-1, keepdim=True)
    var = torch.clamp((x * x).mean(-1, keepdim=True) - mean * mean, min=0.0)
    return (x - mean) / torch.sqrt(var + eps) * p["scale"] + p["bias"]


def mlp_head(x, p):
    for i in range(2):
        ln = p[f"LayerNorm_{i}"]
        x = _ln_relu(layernorm(dense(x, p[f"Dense_{i}"]), ln), ln)
    return x


def _ln_relu(pre, ln):
    """relu of a LayerNorm output; under GATE_MODE the gates of outputs within GATE_TAU_LN (|scale| + |bias|) of
    zero (normalised scale: the forward's accumulated fp32 deviation, amplified by 1/std) are forced."""
    if GATE_MODE is None:
        return torch.relu(pre)
    with torch.no_grad():
        amb = pre.abs() <= GATE_TAU_LN * (ln["scale"].abs() + ln["bias"].abs())
        _gate_count(amb)
    forced = pre if GATE_MODE == "on" else pre * 0.0
    return torch.where(amb, forced, torch.relu(pre))


def gru_cell(p, h, x):
    r = torch.sigmoid(dense(x, p["ir"]) + dense(h, p["hr"]))
    z = torch.sigmoid(dense(x, p["iz"]) + dense(h, p["hz"]))
    n = torch.tanh(dense(x, p["in"]) + r * dense(h, p["hn"]))
    return (1.0 - z) * n + z * h


def lstm_cell(p, c, h, x):
    """flax.linen.LSTMCell: input Denses ii/if/ig/io without bias, hidden Denses hi/hf/hg/ho with bias;
    i, f, o sigmoid, g tanh; c' = f c + i g, h' = o tanh(c').  Returns (c', h')."""
    i = torch.sigmoid(dense(x, p["ii"]) + dense(h, p["hi"]))
    f = torch.sigmoid(dense(x, p["if"]) + dense(h, p["hf"]))
    g = torch.tanh(dense(x, p["ig"]) + dense(h, p["hg"]))
    o = torch.sigmoid(dense(x, p["io"]) + dense(h, p["ho"]))
    c2 = f * c + i * g
    return c2, o * torch.tanh(c2)


def rnn(p, h, x):
    """RNN(rnn_cls, rnn_layers) (dgppo/nn/rnn.py:15-30) on carries h (..., layers * carries * 64), the reference's
    (layers, carries, 64) per agent flattened: returns (the last layer's output, new carries).  p: one GRUCell
    tree (the 1-layer GRU default), a list of GRUCell / LSTMCell trees (carry [c, h] per LSTM layer, the
    reference's jnp.stack((c, h), axis=1)), or [] (use_rnn=False: x passes through, the carry is kept)."""
    if isinstance(p, dict):
        h2 = gru_cell(p, h, x)
        return h2, h2
    if len(p) == 0:
        return x, h
    outs, off = [], 0
    for cell in p:
        if "ii" in cell:
            c2, x = lstm_cell(cell, h[..., off:off + 64], h[..., off + 64:off + 128], x)
            outs += [c2, x]
            off += 128
        else:
            x = gru_cell(cell, h[..., off:off + 64], x)
            outs.append(x)
            off += 64
    return x, torch.cat(outs, -1)


def rnn_width(p, layers=1):
    """carry floats per row for the RNN tree p (no RNN: the reference's unused (layers, 1, 64) zero carry)."""
    if isinstance(p, dict):
        return 64
    if len(p) == 0:
        return 64 * layers
    return sum(128 if "ii" in c else 64 for c in p)


def segment_softmax(logits, seg, num):
    idx = seg[:, None].expand_as(logits)
    mx = torch.full((num,) + logits.shape[1:], -math.inf, dtype=logits.dtype).scatter_reduce(
        0, idx, logits, reduce="amax", include_self=True)
    ex = torch.exp(logits - mx[seg].detach())
    den = torch.zeros((num,) + logits.shape[1:], dtype=logits.dtype).index_add(0, seg, ex)
    return ex / den[seg]


def graph_transformer(p, nodes, edges, recv, send, n_heads, out_dim):
    N = nodes.shape[0]
    xs, xr = nodes[send], nodes[recv]
    q = dense(xr, p["Dense_0"]).reshape(-1, n_heads, out_dim)
    k = dense(xs, p["Dense_1"]).reshape(-1, n_heads, out_dim)
    v = dense(xs, p["Dense_2"]).reshape(-1, n_heads, out_dim)
    e = (edges @ p["Dense_3"]["kernel"]).reshape(-1, n_heads, out_dim)
    attn = (q * k).sum(-1) / math.sqrt(out_dim)
    attn = segment_softmax(attn, recv, N)[..., None]
    msgs = (attn * (v + e)).mean(dim=1)
    agg = torch.zeros((N, out_dim), dtype=nodes.dtype).index_add(0, recv, msgs)
    return _gnn_relu(dense(nodes, p["Dense_4"]) + agg, nodes, p["Dense_4"])


def gnn(layers, graph, n_agents, out_dim=64, msg_dim=32, n_heads=3):
    """GraphTransformerGNN + type_nodes(agent) over a batch of G graphs, evaluated as ONE disjoint
    union graph (node ids offset by g * N): segment softmax / segment sum never cross graphs, so this
    is the per-graph computation of gnn.py:133-142 vmapped, as XLA runs it."""
    nodes = torch.as_tensor(graph["nodes"], dtype=T64)
    edges = torch.as_tensor(graph["edges"], dtype=T64)
    G, N = nodes.shape[:2]
    off = (torch.arange(G, dtype=torch.long) * N)[:, None]
    recv = (torch.as_tensor(graph["receivers"]).long() + off).reshape(-1)
    send = (torch.as_tensor(graph["senders"]).long() + off).reshape(-1)
    x = nodes.reshape(G * N, -1)
    e = edges.reshape(-1, edges.shape[-1])
    L = len(layers)
    for i in range(L):
        od = out_dim if i == L - 1 else msg_dim
        x = graph_transformer(layers[i], x, e, recv, send, n_heads, od)
    return x.reshape(G, N, -1)[:, :n_agents]


STD_INIT_INV = math.log(math.exp(0.5) - 1.0)
THRESH = 0.999


def policy_dist(p, h2):
    feats = dense(h2, p["ScaleHid"])
    means = dense(feats, p["OutputDenseMean"])
    stds = torch.nn.functional.softplus(dense(feats, p["OutputDenseStdTrans"]) + STD_INIT_INV) + 1e-5
    return means, stds


def tanh_fldj(x):
    return 2.0 * (math.log(2.0) - x - torch.nn.functional.softplus(-2.0 * x))


def tanh_normal_log_prob(a, mu, sd):
    inv_t = math.atanh(THRESH)
    log_eps = math.log(1.0 - THRESH)
    left = torch.special.log_ndtr((-inv_t - mu) / sd) - log_eps
    right = torch.special.log_ndtr((mu - inv_t) / sd) - log_eps
    v = torch.clamp(torch.as_tensor(a, dtype=T64), -THRESH, THRESH)
    x = torch.atanh(v)
    z = (x - mu) / sd
    inner = -0.5 * z * z - torch.log(sd) - 0.5 * math.log(2 * math.pi) - tanh_fldj(x)
    lp = torch.where(v <= -THRESH, left, torch.where(v >= THRESH, right, inner))
    return lp.sum(-1)


def tanh_normal_entropy(mu, sd, eps_fixed):
    ent = 0.5 + 0.5 * math.log(2 * math.pi) + torch.log(sd)
    return (ent + tanh_fldj(mu + sd * torch.as_tensor(eps_fixed, dtype=T64))).sum(-1)


def actor_eval_seq(p, graph, S, L, n, actions, eps_fixed):
    """scan_eval_action over S sequences of L graphs (zero carries); graph batch ordered (s, t).
    Returns log_pi, entropy (S, L, n)."""
    y = mlp_head(gnn(p["gnn"], graph, n), p["head"]).reshape(S, L, n, 64)
    h = torch.zeros((S, n, rnn_width(p["gru"])), dtype=T64)
    hs = []
    for t in range(L):
        o, h = rnn(p["gru"], h, y[:, t])
        hs.append(o)
    H = torch.stack(hs, 1)
    mu, sd = policy_dist(p, H)
    act = torch.as_tensor(actions, dtype=T64).reshape(S, L, n, -1)
    return tanh_normal_log_prob(act, mu, sd), tanh_normal_entropy(mu, sd, eps_fixed)


def vl_seq(p, graph, S, L, n, h0=None, return_h=False):
    """scan_Vl over S sequences of L graphs (zero carries unless h0 (S, 64)): values (S, L)."""
    y = mlp_head(gnn(p["gnn"], graph, n).mean(1), p["head"]).reshape(S, L, 64)
    h = torch.zeros((S, rnn_width(p["gru"])), dtype=T64) if h0 is None else torch.as_tensor(h0, dtype=T64)
    vs = []
    for t in range(L):
        o, h = rnn(p["gru"], h, y[:, t])
        vs.append(dense(o, p["out"])[:, 0])
    v = torch.stack(vs, 1)
    return (v, h) if return_h else v


def vh_global_seq(p, graph, S, L, n, h0=None, return_h=False):
    """scan_Vh of InforMARL-Lagr's ValueNet(decompose=True, use_global_info=True) (DecRStateFn,
    value.py:47-79) over S sequences of L graphs, zero carries unless h0 (S, n, 64): values (S, L, n, n_out)."""
    x = gnn(p["gnn"], graph, n)  # (G, n, 64)
    x = torch.cat([x, x.mean(1, keepdim=True).expand(-1, n, -1)], -1)
    y = mlp_head(x, p["head"]).reshape(S, L, n, 64)
    h = torch.zeros((S, n, rnn_width(p["gru"])), dtype=T64) if h0 is None else torch.as_tensor(h0, dtype=T64)
    vs = []
    for t in range(L):
        o, h = rnn(p["gru"], h, y[:, t])
        vs.append(dense(o, p["out"]))
    v = torch.stack(vs, 1)
    return (v, h) if return_h else v


def actor_carry(p, graph, h, n):
    """act(): the policy RNN carry after one graph (policy.py:61-74), h (G, n, W)."""
    y = mlp_head(gnn(p["gnn"], graph, n), p["head"])
    return rnn(p["gru"], torch.as_tensor(h, dtype=T64), y)[1]


def vh(p, graph, h, n):
    y = mlp_head(gnn(p["gnn"], graph, n), p["head"])
    return dense(rnn(p["gru"], torch.as_tensor(h, dtype=T64), y)[0], p["out"])


def ppo_loss(log_pis, log_pis_old, A, entropy, clip_eps=0.25, coef_ent=1e-2):
    ratio = torch.exp(log_pis - torch.as_tensor(log_pis_old, dtype=T64))
    A = torch.as_tensor(A, dtype=T64)
    l1 = -ratio * A
    l2 = -torch.clamp(ratio, 1 - clip_eps, 1 + clip_eps) * A
    return torch.maximum(l1, l2).mean() - coef_ent * entropy.mean()


def grads(tree):
    if isinstance(tree, dict):
        return {k: grads(v) for k, v in tree.items()}
    if isinstance(tree, list):
        return [grads(v) for v in tree]
    return None if tree.grad is None else tree.grad.detach().numpy()


# ---- one DGPPO update (dgppo.py:136-321, informarl.py:357-457) ---------------------------------
def _flat(graph, envs=None):
    """(B, T, ...) host graph dict -> (B*T, ...) env-major (= chunk-major for any rnn_step)."""
    out = {}
    for k in ("nodes", "edges", "receivers", "senders"):
        x = np.asarray(graph[k])
        if envs is not None:
            x = x[envs]
        out[k] = x.reshape((-1,) + x.shape[2:])
    return out


def dgppo_prepass(pa, pl, ph, roll, det, n, dt, gamma, lam, alpha, cbf_eps, cbf_w):
    """Vl / Vh / Dec-OCP GAE / merged advantage of DGPPO.update_inner (dgppo.py:200-283).
    roll / det: dicts of host arrays: graph (B, T, ...) dict, last (B, ...) dict (next_graph[:, -1]),
    rewards (B, T), costs (B, T, n, nh), rnn (B, T, n, 64) stored actor carries."""
    from .nets import compute_dec_ocp_gae
    B, T = roll["rewards"].shape
    with torch.no_grad():
        v, hT = vl_seq(pl, _flat(roll["graph"]), B, T, n, return_h=True)
        vf = vl_seq(pl, _flat({k: x[:, None] for k, x in roll["last"].items()}), B, 1, n, h0=hT)
        Vl = torch.cat([v, vf], 1).numpy()

        def vh_all(r):
            nh = r["costs"].shape[-1]
            vhs = vh(ph, _flat(r["graph"]), np.asarray(r["rnn"]).reshape(B * T, n, -1), n).reshape(B, T, n, nh)
            h2 = actor_carry(pa, _flat({k: x[:, None] for k, x in r["last"].items()}), r["rnn"][:, -1], n)
            vfin = vh(ph, _flat({k: x[:, None] for k, x in r["last"].items()}), h2.numpy(), n)
            return torch.cat([vhs, vfin.reshape(B, 1, n, nh)], 1).numpy()

        Vh, Vh_det = vh_all(roll), vh_all(det)
    Qh, Ql, Qh_det = [], [], []
    for b in range(B):
        qh, ql = compute_dec_ocp_gae(roll["costs"][b].astype(np.float64), -roll["rewards"][b].astype(np.float64),
                                     Vh[b], Vl[b], gamma, lam)
        qhd, _ = compute_dec_ocp_gae(det["costs"][b].astype(np.float64), -det["rewards"][b].astype(np.float64),
                                     Vh_det[b], Vl[b], gamma, lam)
        Qh.append(qh), Ql.append(ql), Qh_det.append(qhd)
    Qh, Ql, Qh_det = np.stack(Qh), np.stack(Ql), np.stack(Qh_det)
    Al = Ql - Vl[:, :T]
    Al = (Al - Al.mean(1, keepdims=True)) / (Al.std(1, keepdims=True) + 1e-8)
    deriv = (Vh[:, 1:] - Vh[:, :T]) / dt + alpha * Vh[:, :T]
    Acbf = np.maximum(deriv + cbf_eps, 0.0)
    is_safe = (deriv <= 0).min(-1)
    A = -(np.where(is_safe, Al[:, :, None], 0.0) + Acbf.max(-1) * cbf_w)
    return dict(Vl=Vl, Vh=Vh, Vh_det=Vh_det, Qh=Qh, Ql=Ql, Qh_det=Qh_det, A=A, deriv=deriv,
                safe_data=is_safe.mean())


def dgppo_minibatch_grads(pa, pl, ph, roll, det, envs, Ql, Qh_det, A, n, L, eps_fixed, clip_eps, coef_ent):
    """Losses + autograd gradients of update_Vl / update_Vh / update_policy for one minibatch of
    envs (targets Ql (B, T), Qh_det (B, T, n, nh) and advantages A (B, T, n) given).  pa/pl/ph must
    be leaf trees with requires_grad."""
    B, T = roll["rewards"].shape
    Bm = len(envs)
    S = Bm * (T // L)
    g = _flat(roll["graph"], envs)
    v = vl_seq(pl, g, S, L, n)
    tgt = torch.as_tensor(Ql[envs].reshape(S, L), dtype=T64)
    loss_vl = (0.5 * (v - tgt) ** 2).mean()
    loss_vl.backward()
    gd = _flat(det["graph"], envs)
    nh = Qh_det.shape[-1]
    out = vh(ph, gd, np.asarray(det["rnn"])[envs].reshape(Bm * T, n, -1), n)
    loss_vh = (0.5 * (out - torch.as_tensor(Qh_det[envs].reshape(Bm * T, n, nh), dtype=T64)) ** 2).mean()
    loss_vh.backward()
    acts = np.asarray(roll["actions"])[envs].reshape(S * L * n, -1)
    lp, ent = actor_eval_seq(pa, g, S, L, n, acts, eps_fixed)
    lp_old = torch.as_tensor(np.asarray(roll["log_pis"])[envs].reshape(S, L, n), dtype=T64)
    adv = torch.as_tensor(A[envs].reshape(S, L, n), dtype=T64)
    loss_pi = ppo_loss(lp, lp_old, adv, ent, clip_eps, coef_ent)
    loss_pi.backward()
    ratio = torch.exp(lp - lp_old).detach()
    return dict(Vl_loss=loss_vl.item(), Vh_loss=loss_vh.item(), policy_loss=loss_pi.item(),
                entropy=ent.mean().item(), tv=0.5 * (ratio - 1).abs().mean().item())

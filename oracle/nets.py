"""NumPy (float64) restatement of the DGPPO networks, distribution, GAE, losses and optimiser.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py; parity unpinned: flax/jraph/tfp/optax are
absent, so their published semantics are restated here and pinned by the KATs in
tests/test_oracle_nets_kat.py).  Parameters use the reference's flax tree layout: every Dense is
{"kernel": (in, out), "bias": (out,)}, kernels act as y = x @ kernel + bias.

Param trees: actor {gnn: [GraphTransformer x2], head, gru, ScaleHid, OutputDenseMean,
OutputDenseStdTrans}; Vl/Vh {gnn, head, gru, out}; GraphTransformer layer {Dense_0 (query),
Dense_1 (key), Dense_2 (value), Dense_3 (edge, no bias), Dense_4 (update)} as flax names them;
gru {ir, iz, in (with bias), hr, hz (no bias), hn (with bias)}.

The GraphTransformer here is the reference's literal per-EDGE form (dgppo/nn/gnn.py:78-117:
gather sender/receiver rows, project per edge, jraph.segment_softmax over receivers, mean over
heads, segment_sum) -- deliberately not the per-receiver algebra the kernels use, so the GPU
path is checked against an independent formulation.
"""
from __future__ import annotations

import numpy as np

D = np.float64


# ---- flax primitives -----------------------------------------------------------------------
def dense(x, p):
    y = x @ p["kernel"]
    if "bias" in p:
        y = y + p["bias"]
    return y


def layernorm(x, p, eps=1e-6):
    """flax.linen.LayerNorm (use_fast_variance): var = E[x^2] - E[x]^2."""
    mean = x.mean(-1, keepdims=True)
    var = np.maximum(0.0, (x * x).mean(-1, keepdims=True) - mean * mean)
    y = (x - mean) / np.sqrt(var + eps)
    return y * p["scale"] + p["bias"]


def relu(x):
    return np.maximum(x, 0.0)


def sigmoid(x):
    return 1.0 / (1.0 + np.exp(-x))


def softplus(x):
    return np.logaddexp(x, 0.0)


def mlp_head(x, p):
    """MLP(hid_sizes=(64, 64), act=relu, act_final=True, layernorm) (dgppo/nn/mlp.py:15-30)."""
    for i in range(2):
        x = relu(layernorm(dense(x, p[f"Dense_{i}"]), p[f"LayerNorm_{i}"]))
    return x


def gru_cell(p, h, x):
    """flax.linen.GRUCell (gate layout ir/iz/in with bias, hr/hz without, hn with bias)."""
    r = sigmoid(dense(x, p["ir"]) + dense(h, p["hr"]))
    z = sigmoid(dense(x, p["iz"]) + dense(h, p["hz"]))
    n = np.tanh(dense(x, p["in"]) + r * dense(h, p["hn"]))
    return (1.0 - z) * n + z * h


# ---- GNN ------------------------------------------------------------------------------------
def segment_softmax(logits, seg, num):
    """jraph.segment_softmax over axis 0 (logits (E, H), seg (E,))."""
    mx = np.full((num,) + logits.shape[1:], -np.inf)
    np.maximum.at(mx, seg, logits)
    ex = np.exp(logits - mx[seg])
    den = np.zeros((num,) + logits.shape[1:])
    np.add.at(den, seg, ex)
    return ex / den[seg]


def graph_transformer(p, nodes, edges, recv, send, n_heads, out_dim):
    """GraphTransformer.__call__ for ONE graph (dgppo/nn/gnn.py:83-117)."""
    N = nodes.shape[0]
    xs, xr = nodes[send], nodes[recv]
    q = dense(xr, p["Dense_0"]).reshape(-1, n_heads, out_dim)
    k = dense(xs, p["Dense_1"]).reshape(-1, n_heads, out_dim)
    v = dense(xs, p["Dense_2"]).reshape(-1, n_heads, out_dim)
    e = (edges @ p["Dense_3"]["kernel"]).reshape(-1, n_heads, out_dim)
    attn = (q * k).sum(-1) / np.sqrt(out_dim)
    attn = segment_softmax(attn, recv, N)[..., None]
    msgs = (attn * (v + e)).mean(axis=1)
    agg = np.zeros((N, out_dim))
    np.add.at(agg, recv, msgs)
    return relu(dense(nodes, p["Dense_4"]) + agg)


def gnn(layers, graph, n_agents, out_dim=64, msg_dim=32, n_heads=3):
    """GraphTransformerGNN (gnn.py:127-142) + type_nodes(0, n) for a batch of graphs.
    layers: list of GraphTransformer param dicts; graph = dict(nodes (G,N,nd), edges (G,E,4),
    receivers, senders (G,E)).  Returns (G, n, out_dim)."""
    out = []
    L = len(layers)
    for g in range(graph["nodes"].shape[0]):
        x = graph["nodes"][g].astype(D)
        for i in range(L):
            od = out_dim if i == L - 1 else msg_dim
            x = graph_transformer(layers[i], x, graph["edges"][g].astype(D),
                                  graph["receivers"][g], graph["senders"][g], n_heads, od)
        out.append(x[:n_agents])  # agent rows come first in every env graph
    return np.stack(out)


# ---- policy / value heads ------------------------------------------------------------------
STD_INIT_INV = np.log(np.exp(0.5) - 1.0)  # TanhNormal.std_dev_init_inv (policy.py:54-59)


def policy_features(p, graph, rnn_state, n_agents):
    """PolicyNet + TanhNormal body (policy.py:25-33, 61-74) for (G,) graphs and rnn_state (G,1,n,1,64).
    p = {gnn: [2 layers], head, gru, ScaleHid, OutputDenseMean, OutputDenseStdTrans}.
    Returns (means (G,n,2), stds (G,n,2), new_rnn_state)."""
    x = gnn(p["gnn"], graph, n_agents)
    x = mlp_head(x, p["head"])
    h = rnn_state[:, 0, :, 0, :]
    h2 = gru_cell(p["gru"], h, x)
    feats = dense(h2, p["ScaleHid"])
    means = dense(feats, p["OutputDenseMean"])
    stds = softplus(dense(feats, p["OutputDenseStdTrans"]) + STD_INIT_INV) + 1e-5
    return means, stds, h2[:, None, :, None, :]


def value_Vl(p, graph, rnn_state, n_agents):
    """RStateFn (value.py:15-44): GNN -> mean over agents -> head -> GRU -> Dense(1).
    rnn_state (G, 1, 1, 1, 64).  Returns (V (G,), new_state)."""
    x = gnn(p["gnn"], graph, n_agents).mean(axis=1)
    x = mlp_head(x, p["head"])
    h2 = gru_cell(p["gru"], rnn_state[:, 0, 0, 0, :], x)
    return dense(h2, p["out"])[:, 0], h2[:, None, None, None, :]


def value_Vh(p, graph, rnn_state, n_agents):
    """DecRStateFn (value.py:47-79), use_global_info=False, 1 GNN layer; rnn_state = the ACTOR's
    carry (G, 1, n, 1, 64).  Returns Vh (G, n, n_cost)."""
    x = gnn(p["gnn"], graph, n_agents)
    x = mlp_head(x, p["head"])
    h2 = gru_cell(p["gru"], rnn_state[:, 0, :, 0, :], x)
    return dense(h2, p["out"])


# ---- TanhTransformedDistribution (distribution.py:10-66) + tfp Normal/Tanh -------------------
THRESH = 0.999


def _log_ndtr(x):
    from scipy.special import log_ndtr

    return log_ndtr(x)


def normal_logpdf(x, mu, sd):
    z = (x - mu) / sd
    return -0.5 * z * z - np.log(sd) - 0.5 * np.log(2 * np.pi)


def tanh_fldj(x):
    """tfb.Tanh.forward_log_det_jacobian: 2 (log 2 - x - softplus(-2x))."""
    return 2.0 * (np.log(2.0) - x - softplus(-2.0 * x))


def tanh_normal_log_prob(a, mu, sd):
    """log_prob of Independent(TanhTransformed(Normal)) summed over the last axis."""
    inv_t = np.arctanh(THRESH)
    log_eps = np.log(1.0 - THRESH)
    left = _log_ndtr((-inv_t - mu) / sd) - log_eps
    right = _log_ndtr(-(inv_t - mu) / sd) - log_eps  # log survival
    v = np.clip(a, -THRESH, THRESH)
    x = np.arctanh(v)
    inner = normal_logpdf(x, mu, sd) - tanh_fldj(x)
    lp = np.where(v <= -THRESH, left, np.where(v >= THRESH, right, inner))
    return lp.sum(-1)


def tanh_normal_entropy(mu, sd, eps_fixed):
    """entropy(): Normal entropy + fldj(mu + sd * eps) with eps a FIXED draw (the reference seeds
    it once at trace time, distribution.py:37-43; identical for every vmapped instance)."""
    ent = 0.5 + 0.5 * np.log(2 * np.pi) + np.log(sd)
    return (ent + tanh_fldj(mu + sd * eps_fixed)).sum(-1)


# ---- GAE (dgppo/algo/utils.py:11-79), literal restatement -----------------------------------
def compute_dec_ocp_gae(Tah_hs, T_l, Tp1ah_Vh, Tp1_Vl, disc_gamma, gae_lambda):
    """The reference scans `inps = (ts = arange(T)[::-1], hs, l, Vh, Vl)` with
    `lax.scan(..., reverse=True)` (utils.py:73-76): the data are visited from time T-1 down to 0 while
    the loop variable `ii` = ts[k] = T-1-k COUNTS the steps taken (0, 1, ..., T-1).  `ii` drives the
    mask (rows 0..ii live) and the coefficient updates; `k` indexes the data and the output.  With this
    reading Ql is exactly the textbook TD(lambda) return of l (tests/test_oracle_kat.py)."""
    T, n_agent, nh = Tah_hs.shape
    Tah_Vh, T_Vl = Tp1ah_Vh[:-1], np.repeat(Tp1_Vl[:-1][:, None], n_agent, axis=1)
    Vh_final, Vl_final = Tp1ah_Vh[-1], Tp1_Vl[-1]
    next_Vhs_row = np.zeros((T + 1, n_agent, nh))
    next_Vhs_row[0] = Vh_final
    next_Vl_row = np.zeros((T + 1, n_agent))
    next_Vl_row[0] = Vl_final
    gae_coeffs = np.zeros(T + 1)
    gae_coeffs[0] = 1.0
    Qs = np.zeros((T, n_agent, nh + 1))
    for k in range(T - 1, -1, -1):  # scan(reverse=True) order over the data
        ii = T - 1 - k  # ts[k]
        hs, l, Vhs, Vl = Tah_hs[k], T_l[k], Tah_Vh[k], T_Vl[k]
        mask = np.arange(T + 1) < ii + 1
        h_disc = hs.max(-1)
        disc_to_h = (1 - disc_gamma) * h_disc[None, :, None] + disc_gamma * next_Vhs_row
        Vhs_row = mask[:, None, None] * np.maximum(hs, disc_to_h)
        Vl_row = mask[:, None] * (l + disc_gamma * next_Vl_row)
        cat = np.concatenate([Vhs_row, Vl_row[:, :, None]], axis=-1)
        Qs[k] = np.einsum("tah,t->ah", cat, gae_coeffs)
        Vhs_row = Vhs_row.copy()
        Vl_row = Vl_row.copy()
        Vhs_row[ii + 1] = Vhs
        Vl_row[ii + 1] = Vl
        gae_coeffs = np.roll(gae_coeffs, 1)
        gae_coeffs[0] = gae_lambda ** (ii + 1)
        gae_coeffs[1] = (gae_lambda ** ii) * (1 - gae_lambda)
        next_Vhs_row, next_Vl_row = Vhs_row, Vl_row
    return Qs[:, :, :nh], Qs[:, 0, nh]


# ---- optimiser (optax.adam + apply_if_finite, trainer/utils.py:105-118) ----------------------
def clip_by_global_norm_ref(grads, max_norm):
    g_norm = np.sqrt(sum((g.astype(D) ** 2).sum() for g in grads))
    scale = max_norm / max(max_norm, g_norm)
    return [g * scale for g in grads], g_norm


def adam_step(params, grads, mu, nu, count, lr, b1=0.9, b2=0.999, eps=1e-8):
    """optax.scale_by_adam + scale(-lr) + apply_updates; count is the pre-increment step count."""
    t = count + 1
    out_p, out_m, out_v = [], [], []
    for p, g, m, v in zip(params, grads, mu, nu):
        m = b1 * m + (1 - b1) * g
        v = b2 * v + (1 - b2) * g * g
        mh = m / (1 - b1 ** t)
        vh = v / (1 - b2 ** t)
        out_p.append(p - lr * mh / (np.sqrt(vh) + eps))
        out_m.append(m)
        out_v.append(v)
    return out_p, out_m, out_v


def ppo_policy_loss(log_pis, log_pis_old, A, entropy, clip_eps=0.25, coef_ent=1e-2):
    """update_policy loss (informarl.py:428-438)."""
    ratio = np.exp(log_pis - log_pis_old)
    l1 = -ratio * A
    l2 = -np.clip(ratio, 1 - clip_eps, 1 + clip_eps) * A
    loss = np.maximum(l1, l2).mean() - coef_ent * entropy.mean()
    return loss, dict(clip_frac=(l2 > l1).mean(), entropy=entropy.mean(),
                      total_variation_dist=0.5 * np.abs(ratio - 1.0).mean())


# ---- InforMARL (dgppo/algo/informarl.py) ------------------------------------------------------------
def informarl_shaped_l(rewards, costs, cost_weight):
    """T_l of informarl.py:329: -reward + w * sum over (agent, cost) of max(cost, 0), (B, T)."""
    r = np.asarray(rewards, np.float64)
    c = np.maximum(np.asarray(costs, np.float64), 0.0)
    return -r + cost_weight * c.sum(-1).sum(-1)


def informarl_advantages(Ql, Vl, n_agents):
    """informarl.py:334-337: Al = Ql - Vl[:, :T] normalised over T per env (population std), A = -Al per agent."""
    Al = np.asarray(Ql, np.float64) - np.asarray(Vl, np.float64)[:, :-1]
    Al = (Al - Al.mean(axis=1, keepdims=True)) / (Al.std(axis=1, keepdims=True) + 1e-8)
    return -np.repeat(Al[:, :, None], n_agents, axis=-1)


def lagr_advantages(Ql, Vl, Qh, Vh, lagr):
    """InforMARL-Lagr (informarl_lagr.py:205-221): Al = Ql - Vl[:, :T] normalised over T per env;
    Ah = Qh - Vh[:, :T] normalised over T per (env, agent, cost); A = -Al - mean_h(Ah * lagr).
    Returns (A (B, T, n), Ah (B, T, n, nh))."""
    Ql, Vl, Qh, Vh, lagr = (np.asarray(x, np.float64) for x in (Ql, Vl, Qh, Vh, lagr))
    T = Ql.shape[1]
    Al = Ql - Vl[:, :T]
    Al = (Al - Al.mean(axis=1, keepdims=True)) / (Al.std(axis=1, keepdims=True) + 1e-8)
    Ah = Qh - Vh[:, :T]
    Ah = (Ah - Ah.mean(axis=1, keepdims=True)) / (Ah.std(axis=1, keepdims=True) + 1e-8)
    return -Al[:, :, None] - (Ah * lagr[None, None]).mean(-1), Ah


def lagr_update(lagr, log_pi, log_pi_old, Vh, Ah, gamma, lr):
    """update_lagr (informarl_lagr.py:283-305): ratio = exp(log_pi - log_pi_old) (B, T, n);
    delta = -mean_{b,t}(Vh (1 - gamma) + ratio Ah) (n, nh); lagr <- relu(lagr - lr delta)."""
    ratio = np.exp(np.asarray(log_pi, np.float64) - np.asarray(log_pi_old, np.float64))
    delta = -(np.asarray(Vh, np.float64) * (1 - gamma) + ratio[..., None] * np.asarray(Ah, np.float64)).mean((0, 1))
    return np.maximum(np.asarray(lagr, np.float64) - delta * lr, 0.0)


def merged_cbf_advantages(Ql, Vl, Vh, n_agents, dt, alpha, cbf_eps, cbf_weight):
    """DGPPO's merged advantage (dgppo.py:239-259, identical in hcbfcrpo.py:163-183): Al = Ql - Vl[:, :T]
    normalised over T; deriv = (Vh[t+1] - Vh[t]) / dt + alpha Vh[t]; Acbf = max(deriv + eps, 0);
    A = -(where(all_h deriv <= 0, Al, 0) + max_h Acbf * w).  Returns (A (B, T, n), safe fraction)."""
    Ql, Vl, Vh = (np.asarray(x, np.float64) for x in (Ql, Vl, Vh))
    T = Ql.shape[1]
    Al = Ql - Vl[:, :T]
    Al = (Al - Al.mean(axis=1, keepdims=True)) / (Al.std(axis=1, keepdims=True) + 1e-8)
    deriv = (Vh[:, 1:] - Vh[:, :T]) / dt + alpha * Vh[:, :T]
    Acbf = np.maximum(deriv + cbf_eps, 0.0)
    safe = (deriv <= 0).min(-1)
    A = -(np.where(safe, np.repeat(Al[:, :, None], n_agents, -1), 0.0) + Acbf.max(-1) * cbf_weight)
    return A, safe.mean(), deriv

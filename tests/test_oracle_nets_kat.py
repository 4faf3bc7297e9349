"""Hand-derived known-answer tests that pin the network half of the oracle (oracle/nets.py and its
float64 autograd twin oracle/nets_t.py) where it restates third-party semantics the reference
calls but does not contain: flax LayerNorm (eps 1e-6, fast variance), flax
GRUCell (gate / bias layout), jraph.segment_softmax, tfp's clipped TanhNormal log-prob and
optax adam + clip_by_global_norm.

Every expected value below is computed from scalar closed forms with the `math` module (not with
the oracle's own vectorised code), so a wrong restatement fails here.  The libraries themselves are
absent, so the KATs pin the oracle to their published definitions: parity stays "unpinned" against
the reference's runtime, but the restated arithmetic is checked by hand."""
import math

import numpy as np
import pytest
import torch

from oracle import nets as O
from oracle import nets_t as R


def _both(fn_np, fn_t, *args):
    """Evaluate an oracle function in its NumPy and torch-float64 forms."""
    a = np.asarray(fn_np(*[np.asarray(x, np.float64) if isinstance(x, (list, np.ndarray)) else x for x in args]))
    b = fn_t(*[torch.as_tensor(np.asarray(x, np.float64)) if isinstance(x, (list, np.ndarray)) else x for x in args])
    return a, b.detach().numpy()


# ---- flax.linen.LayerNorm (mlp.py:27: nn.LayerNorm(), epsilon 1e-6, scale + bias) ------------------
def test_layernorm_hand_values():
    x = [1.0, 2.0, 3.0, 4.0]
    mean = 2.5
    var = (1 + 4 + 9 + 16) / 4 - mean * mean  # fast variance E[x^2] - E[x]^2 = 1.25
    scale, bias = [1.0, 2.0, 0.5, -1.0], [0.0, 0.1, -0.2, 0.3]
    want = [(xi - mean) / math.sqrt(var + 1e-6) * s + b for xi, s, b in zip(x, scale, bias)]
    p = {"scale": np.array(scale), "bias": np.array(bias)}
    got = O.layernorm(np.array([x]), p)[0]
    np.testing.assert_allclose(got, want, rtol=0, atol=1e-14)
    got_t = R.layernorm(torch.tensor([x], dtype=torch.float64), R.to_t(p))[0].numpy()
    np.testing.assert_allclose(got_t, want, rtol=0, atol=1e-14)


def test_layernorm_constant_row_uses_eps():
    # var = 0: y = (x - mean) / sqrt(1e-6) = 0 exactly, output = bias
    p = {"scale": np.ones(3), "bias": np.array([0.5, -0.5, 2.0])}
    np.testing.assert_array_equal(O.layernorm(np.full((1, 3), 7.0), p)[0], [0.5, -0.5, 2.0])
    # a tiny spread is scaled by 1/sqrt(var + 1e-6), not 1/sqrt(var)
    x = np.array([[0.0, 1e-3]])
    want = 5e-4 / math.sqrt(2.5e-7 + 1e-6)
    np.testing.assert_allclose(O.layernorm(x, {"scale": np.ones(2), "bias": np.zeros(2)})[0], [-want, want],
                               rtol=1e-12)


# ---- flax.linen.GRUCell (rnn.py:15-30) -------------------------------------------------------------
def _sig(v):
    return 1.0 / (1.0 + math.exp(-v))


def test_grucell_gate_layout_hand_values():
    """flax GRUCell: r = s(W_ir x + b_ir + W_hr h), z = s(W_iz x + b_iz + W_hz h),
    n = tanh(W_in x + b_in + r * (W_hn h + b_hn)), h' = (1 - z) n + z h; hr / hz have no bias."""
    x, h = 0.5, 0.25
    w = dict(ir=1.0, bir=0.0, hr=1.0, iz=-1.0, biz=0.5, hz=2.0, in_=2.0, bin=0.1, hn=3.0, bhn=-0.2)
    r = _sig(w["ir"] * x + w["bir"] + w["hr"] * h)
    z = _sig(w["iz"] * x + w["biz"] + w["hz"] * h)
    n = math.tanh(w["in_"] * x + w["bin"] + r * (w["hn"] * h + w["bhn"]))
    want = (1 - z) * n + z * h
    k = lambda v: np.array([[v]])  # noqa: E731
    b = lambda v: np.array([v])  # noqa: E731
    p = {"ir": {"kernel": k(w["ir"]), "bias": b(w["bir"])}, "iz": {"kernel": k(w["iz"]), "bias": b(w["biz"])},
         "in": {"kernel": k(w["in_"]), "bias": b(w["bin"])}, "hr": {"kernel": k(w["hr"])},
         "hz": {"kernel": k(w["hz"])}, "hn": {"kernel": k(w["hn"]), "bias": b(w["bhn"])}}
    got = O.gru_cell(p, np.array([[h]]), np.array([[x]]))[0, 0]
    assert abs(got - want) < 1e-15
    got_t = R.gru_cell(R.to_t(p), torch.tensor([[h]], dtype=torch.float64), torch.tensor([[x]], dtype=torch.float64))
    assert abs(got_t.item() - want) < 1e-15
    # b_hn sits INSIDE the reset product: moving it to b_in changes the answer
    n_wrong = math.tanh(w["in_"] * x + w["bin"] + w["bhn"] + r * (w["hn"] * h))
    assert abs(((1 - z) * n_wrong + z * h) - want) > 1e-3


def test_grucell_zero_weights_halves_carry():
    z64 = {"kernel": np.zeros((2, 2)), "bias": np.zeros(2)}
    p = {"ir": z64, "iz": z64, "in": z64, "hr": {"kernel": np.zeros((2, 2))}, "hz": {"kernel": np.zeros((2, 2))},
         "hn": z64}
    h = np.array([[0.8, -2.0]])
    np.testing.assert_array_equal(O.gru_cell(p, h, np.array([[3.0, 4.0]])), 0.5 * h)  # r = z = 0.5, n = 0


def test_lstmcell_hand_values():
    """flax LSTMCell (--use-lstm): i/f/o = sigmoid, g = tanh of (x W_i* + h W_h* + b_h*), the input Denses have
    no bias; c' = f c + i g, h' = o tanh(c')."""
    x, c, h = 0.5, -0.3, 0.25
    w = dict(ii=1.0, hi=0.5, bi=0.1, if_=-1.0, hf=2.0, bf=0.3, ig=2.0, hg=-1.5, bg=-0.2, io=0.7, ho=1.1, bo=0.0)
    i = _sig(w["ii"] * x + w["hi"] * h + w["bi"])
    f = _sig(w["if_"] * x + w["hf"] * h + w["bf"])
    g = math.tanh(w["ig"] * x + w["hg"] * h + w["bg"])
    o = _sig(w["io"] * x + w["ho"] * h + w["bo"])
    c_want = f * c + i * g
    h_want = o * math.tanh(c_want)
    k = lambda v: torch.tensor([[v]], dtype=torch.float64)  # noqa: E731
    b = lambda v: torch.tensor([v], dtype=torch.float64)  # noqa: E731
    p = {"ii": {"kernel": k(w["ii"])}, "if": {"kernel": k(w["if_"])}, "ig": {"kernel": k(w["ig"])},
         "io": {"kernel": k(w["io"])}, "hi": {"kernel": k(w["hi"]), "bias": b(w["bi"])},
         "hf": {"kernel": k(w["hf"]), "bias": b(w["bf"])}, "hg": {"kernel": k(w["hg"]), "bias": b(w["bg"])},
         "ho": {"kernel": k(w["ho"]), "bias": b(w["bo"])}}
    c2, h2 = R.lstm_cell(p, k(c), k(h), k(x))
    assert abs(c2.item() - c_want) < 1e-15 and abs(h2.item() - h_want) < 1e-15
    # the stacked form: carry rows [c | h] (64 wide per carry), two layers, the second fed the first's h'
    H = 64
    z = lambda *sh: torch.zeros(sh, dtype=torch.float64)  # noqa: E731
    cell = {key: ({"kernel": z(H, H)} if key[0] == "i" else {"kernel": z(H, H), "bias": z(H)})
            for key in ("ii", "if", "ig", "io", "hi", "hf", "hg", "ho")}
    carry = torch.cat([torch.full((1, H), 2.0, dtype=torch.float64), z(1, H), torch.full((1, H), -4.0, dtype=torch.float64),
                       z(1, H)], 1)
    out, new = R.rnn([cell, cell], carry, z(1, H))
    # zero weights: i = f = o = 1/2, g = 0 -> c' = c / 2, h' = tanh(c') / 2 per layer
    assert R.rnn_width([cell, cell]) == 4 * H and new.shape == (1, 4 * H)
    np.testing.assert_allclose(new[0, :H].numpy(), 1.0)
    np.testing.assert_allclose(new[0, H:2 * H].numpy(), 0.5 * math.tanh(1.0))
    np.testing.assert_allclose(new[0, 2 * H:3 * H].numpy(), -2.0)
    np.testing.assert_allclose(out[0].numpy(), 0.5 * math.tanh(-2.0))
    # no RNN: features pass through, the carry is kept
    o2, c2n = R.rnn([], carry, torch.ones((1, H), dtype=torch.float64))
    assert torch.equal(o2, torch.ones((1, H), dtype=torch.float64)) and torch.equal(c2n, carry)


# ---- jraph.segment_softmax / GraphTransformer (gnn.py:99-117) ----------------------------------------
def test_segment_softmax_uniform_logits_give_inverse_in_degree():
    seg = np.array([0, 0, 0, 2, 2, 1])  # in-degrees 3, 1, 2
    a, b = _both(lambda l: O.segment_softmax(l, seg, 4), lambda l: R.segment_softmax(l, torch.as_tensor(seg), 4),
                 np.zeros((6, 3)))
    want = np.array([1 / 3, 1 / 3, 1 / 3, 1 / 2, 1 / 2, 1.0])[:, None].repeat(3, 1)
    np.testing.assert_allclose(a, want, atol=1e-15)
    np.testing.assert_allclose(b, want, atol=1e-15)


def test_segment_softmax_hand_values_and_shift_invariance():
    seg = np.array([0, 0])
    logits = np.array([[0.0], [math.log(3.0)]])
    np.testing.assert_allclose(O.segment_softmax(logits, seg, 1)[:, 0], [0.25, 0.75], atol=1e-15)
    # max-shifted: huge logits do not overflow
    np.testing.assert_allclose(O.segment_softmax(logits + 1000.0, seg, 1)[:, 0], [0.25, 0.75], atol=1e-15)


def test_graph_transformer_uniform_attention_hand_values():
    """q = 0 (Dense_0 zero) -> every logit 0 -> attention 1/in-degree; v = x_send (Dense_2 = 1),
    no edge term, no update term: out_i = relu(mean over in-edges of x_send).  Edges (recv <- send):
    0 <- 1, 0 <- 2, 1 <- 2; node 2 receives nothing."""
    nodes = np.array([[1.0], [2.0], [4.0]])
    edges = np.zeros((3, 4))
    recv, send = np.array([0, 0, 1]), np.array([1, 2, 2])
    one = {"kernel": np.ones((1, 1)), "bias": np.zeros(1)}
    zero = {"kernel": np.zeros((1, 1)), "bias": np.zeros(1)}
    p = {"Dense_0": zero, "Dense_1": one, "Dense_2": one, "Dense_3": {"kernel": np.zeros((4, 1))}, "Dense_4": zero}
    want = [[(2.0 + 4.0) / 2], [4.0], [0.0]]
    np.testing.assert_allclose(O.graph_transformer(p, nodes, edges, recv, send, 1, 1), want, atol=1e-15)
    got_t = R.graph_transformer(R.to_t(p), torch.as_tensor(nodes), torch.as_tensor(edges), torch.as_tensor(recv),
                                torch.as_tensor(send), 1, 1)
    np.testing.assert_allclose(got_t.numpy(), want, atol=1e-15)


def test_graph_transformer_heads_are_averaged():
    """Two heads with v = +x and v = 3x: messages are the MEAN over heads (gnn.py:111), = 2x."""
    nodes = np.array([[0.0], [1.5]])
    recv, send = np.array([0]), np.array([1])
    p = {"Dense_0": {"kernel": np.zeros((1, 2)), "bias": np.zeros(2)},
         "Dense_1": {"kernel": np.ones((1, 2)), "bias": np.zeros(2)},
         "Dense_2": {"kernel": np.array([[1.0, 3.0]]), "bias": np.zeros(2)},
         "Dense_3": {"kernel": np.zeros((4, 2))}, "Dense_4": {"kernel": np.zeros((1, 1)), "bias": np.zeros(1)}}
    out = O.graph_transformer(p, nodes, np.zeros((1, 4)), recv, send, 2, 1)
    np.testing.assert_allclose(out[:, 0], [3.0, 0.0], atol=1e-15)


# ---- tfp TanhTransformedDistribution log-prob (distribution.py:25-35) --------------------------------
def _log_phi(x):  # log of the standard normal CDF via erfc (independent of scipy / torch log_ndtr)
    return math.log(0.5 * math.erfc(-x / math.sqrt(2.0)))


@pytest.mark.parametrize("mu,sd", [(0.0, 1.0), (0.3, 0.5), (-1.2, 2.0)])
def test_tanh_normal_log_prob_clip_edges(mu, sd):
    inv_t = math.atanh(0.999)
    left = _log_phi((-inv_t - mu) / sd) - math.log(1e-3)  # log_cdf(-atanh .999) - log(1 - .999)
    right = _log_phi((mu - inv_t) / sd) - math.log(1e-3)  # log_survival(atanh .999) - log(1 - .999)
    for a, want in ((-1.0, left), (-0.9995, left), (1.0, right), (0.99999, right)):
        got = O.tanh_normal_log_prob(np.array([[a]]), np.array([[mu]]), np.array([[sd]]))[0]
        assert abs(got - want) < 1e-10, (a, got, want)
        got_t = R.tanh_normal_log_prob(np.array([[a]]), torch.tensor([[mu]], dtype=torch.float64),
                                       torch.tensor([[sd]], dtype=torch.float64))[0].item()
        assert abs(got_t - want) < 1e-10, (a, got_t, want)


def test_tanh_normal_log_prob_interior_hand_values():
    # a = tanh(1), N(0, 1): log N(1) - log(1 - tanh(1)^2)
    a = math.tanh(1.0)
    want = -0.5 - 0.5 * math.log(2 * math.pi) - math.log(1 - a * a)
    got = O.tanh_normal_log_prob(np.array([[a]]), np.zeros((1, 1)), np.ones((1, 1)))[0]
    assert abs(got - want) < 1e-9
    # summed over the action dim (Independent): two components add
    got2 = O.tanh_normal_log_prob(np.array([[0.0, a]]), np.zeros((1, 2)), np.ones((1, 2)))[0]
    assert abs(got2 - (want - 0.5 * math.log(2 * math.pi))) < 1e-9


def test_tanh_fldj_is_log_one_minus_tanh_squared():
    for x in (-3.0, -0.2, 0.0, 0.7, 5.0):
        assert abs(O.tanh_fldj(x) - math.log(1 - math.tanh(x) ** 2)) < 1e-9


# ---- optax adam + clip_by_global_norm + apply_if_finite (informarl.py:131-137, trainer/utils.py:105-118) --
def test_adam_one_step_on_quadratic():
    """f(p) = 0.5 c p^2, g = c p.  Step 1: m = 0.1 g, v = 0.001 g^2, m_hat = g, v_hat = g^2, so
    p1 = p0 - lr g / (|g| + eps)."""
    c, lr = 3.0, 1e-3
    p0 = np.array([2.0, -0.5, 1e-9])
    g = c * p0
    (p1,), (m1,), (v1,) = O.adam_step([p0], [g], [np.zeros(3)], [np.zeros(3)], 0, lr)
    want = [pi - lr * gi / (abs(gi) + 1e-8) for pi, gi in zip(p0, g)]
    np.testing.assert_allclose(p1, want, rtol=0, atol=1e-15)
    np.testing.assert_allclose(m1, 0.1 * g, rtol=1e-15)
    np.testing.assert_allclose(v1, 0.001 * g * g, rtol=1e-15)
    # step 2 by hand on the new gradient
    g2 = c * p1
    m2, v2 = 0.9 * m1 + 0.1 * g2, 0.999 * v1 + 0.001 * g2 * g2
    want2 = p1 - lr * (m2 / (1 - 0.9 ** 2)) / (np.sqrt(v2 / (1 - 0.999 ** 2)) + 1e-8)
    (p2,), _, _ = O.adam_step([p1], [g2], [m1], [v1], 1, lr)
    np.testing.assert_allclose(p2, want2, rtol=0, atol=1e-15)


def test_clip_by_global_norm_hand_values():
    g = [np.array([3.0, 0.0]), np.array([4.0])]  # global norm 5
    (a, b), n = O.clip_by_global_norm_ref(g, 2.0)
    assert n == 5.0
    np.testing.assert_allclose(np.concatenate([a, b]), [1.2, 0.0, 1.6], atol=1e-15)
    (a, b), n = O.clip_by_global_norm_ref([np.array([0.3]), np.array([0.4])], 2.0)  # below the limit: unchanged
    np.testing.assert_allclose([a[0], b[0]], [0.3, 0.4], atol=1e-15)


# ---- PPO loss (informarl.py:428-438) -----------------------------------------------------------------------
def test_ppo_clipped_loss_hand_values():
    lp_old = np.zeros(3)
    lp = np.array([math.log(1.5), math.log(0.5), 0.0])  # ratios 1.5 (clipped to 1.25), 0.5 (clipped 0.75), 1
    A = np.array([1.0, -2.0, 0.5])
    ent = np.array([0.2, 0.4, 0.6])
    # max(-r A, -clip(r) A): [-1.25, 1.5, -0.5] -> mean -1/12; minus 0.01 * mean entropy 0.4
    loss, info = O.ppo_policy_loss(lp, lp_old, A, ent)
    assert abs(loss - (-1.0 / 12 - 0.004)) < 1e-12
    assert abs(info["clip_frac"] - 2 / 3) < 1e-12
    assert abs(info["total_variation_dist"] - 0.5 * (0.5 + 0.5 + 0.0) / 3) < 1e-12


def test_lagr_advantages_and_update_kat():
    """InforMARL-Lagr by hand (informarl_lagr.py:205-221, 283-305): Ql - Vl = [0, 2] per env normalises to
    [-1, 1]; Qh - Vh = [1, 3] likewise; A = -Al - mean_h(Ah lagr). With log pi = old log pi (ratio 1),
    Vh = c and Ah with zero mean over (b, t), delta = -c (1 - gamma): lagr + lr c (1 - gamma)."""
    Ql = np.array([[0.0, 2.0]])
    Vl = np.zeros((1, 3))
    Qh = np.array([[1.0, 3.0]])[:, :, None, None] * np.ones((1, 2, 1, 2))
    Vh = np.zeros((1, 3, 1, 2))
    lagr = np.array([[0.5, 1.5]])
    A, Ah = O.lagr_advantages(Ql, Vl, Qh, Vh, lagr)
    np.testing.assert_allclose(Ah[0, :, 0, 0], [-1.0, 1.0], atol=1e-7)
    np.testing.assert_allclose(A[0, :, 0], [1.0 + 1.0, -1.0 - 1.0], atol=1e-7)  # mean_h(lagr) = 1
    lp = np.zeros((1, 2, 1))
    out = O.lagr_update(lagr, lp, lp, np.full((1, 2, 1, 2), 3.0), Ah, 0.9, 0.1)
    np.testing.assert_allclose(out, lagr + 0.1 * 3.0 * 0.1, atol=1e-12)
    # relu: a large negative Vh drives the multiplier to zero
    out = O.lagr_update(lagr, lp, lp, np.full((1, 2, 1, 2), -1e3), Ah, 0.9, 0.1)
    assert (out == 0).all()

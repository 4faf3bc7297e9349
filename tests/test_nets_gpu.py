"""GPU parity for hot path (2): the MFMA GEMM, and the actor / Vl / Vh networks (forward AND
gradients) against the float64 per-edge reference formulation (oracle/nets_t.py, autograd).

Tolerances (fp32 kernels vs float64 reference): forward outputs |gpu - ref| <= 1e-5 + 1e-5 |ref|;
gradients |gpu - ref| <= 2e-5 * max|ref| + 1e-6 per parameter tensor (the kernels use a different
but algebraically identical per-receiver formulation and different summation orders)."""
import numpy as np
import pytest
import torch

from dgppo_fov_amd.algo.module.nets import ActorNet, VhNet, VlNet
from dgppo_fov_amd.env import make_env
from dgppo_fov_amd.nn import kernels as K
from dgppo_fov_amd.nn.layers import GraphBatch
from oracle import nets_t as R

pytestmark = pytest.mark.gpu


def _close(a, b, rtol=1e-5, atol=1e-5, what=""):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    err = np.abs(a - b) - (atol + rtol * np.abs(b))
    assert err.max() <= 0, f"{what}: max excess {err.max():.3e}, max abs err {np.abs(a - b).max():.3e}"


def _grad_close(g, r, what):
    g = np.asarray(g, np.float64)
    r = np.asarray(r, np.float64)
    scale = np.abs(r).max()
    err = np.abs(g - r).max()
    assert err <= 2e-5 * scale + 1e-6, f"{what}: max abs err {err:.3e} vs scale {scale:.3e}"


def _walk(a, b, path=""):
    if isinstance(a, dict):
        for k in a:
            yield from _walk(a[k], b[k], f"{path}/{k}")
    elif isinstance(a, list):
        for i, (x, y) in enumerate(zip(a, b)):
            yield from _walk(x, y, f"{path}[{i}]")
    else:
        yield path, a, b


# ---- GEMM ------------------------------------------------------------------------------------
@pytest.mark.parametrize("M,N,Kd,ta,tb,batch", [(1, 1, 1, 0, 0, 1), (70, 33, 17, 0, 0, 1), (64, 64, 64, 1, 0, 1),
                                               (130, 5, 200, 0, 1, 1), (7, 96, 3000, 1, 0, 1),
                                               (50, 40, 20, 1, 1, 3), (33, 192, 9000, 1, 0, 2)])
def test_gemm_matches_float64(cuda, M, N, Kd, ta, tb, batch):
    g = torch.Generator().manual_seed(M * 7 + N)
    A = torch.randn(batch, *((Kd, M) if ta else (M, Kd)), generator=g, dtype=torch.float64)
    B = torch.randn(batch, *((N, Kd) if tb else (Kd, N)), generator=g, dtype=torch.float64)
    C0 = torch.randn(batch, M, N, generator=g, dtype=torch.float64)
    bias = torch.randn(N, generator=g, dtype=torch.float64)
    opA = A.transpose(1, 2) if ta else A
    opB = B.transpose(1, 2) if tb else B
    ref = torch.relu(0.5 * opA @ opB + 0.25 * C0 + bias)
    Ad, Bd, Cd = A.float().to(cuda), B.float().to(cuda), C0.float().to(cuda).contiguous()
    K.gemm(Ad, Bd, Cd, M, N, Kd, ta=bool(ta), tb=bool(tb), batch=batch, sa=A[0].numel(), sb=B[0].numel(),
           sc=M * N, bias=bias.float().to(cuda), alpha=0.5, beta=0.25, relu=True)
    torch.cuda.synchronize()
    scale = (opA.abs() @ opB.abs()).max().item()
    assert (Cd.double().cpu() - ref).abs().max().item() <= 2e-6 * scale + 1e-5


@pytest.mark.parametrize("M,N,Kd,batch,grp", [(64, 192, 131072, 1, 0), (111, 64, 20000, 1, 0), (7, 32, 70001, 1, 0),
                                               (64, 32, 5000, 3, 0), (200, 150, 3001, 1, 0), (64, 192, 4096, 1, 24),
                                               (36, 64, 777, 2, 7)])
def test_gemm_weight_grad_with_fused_bias_grad(cuda, M, N, Kd, batch, grp):
    """dW = A^T B (+ beta) with db = colsum(B) fused (the wgrad path), incl. row-grouped operands."""
    g = torch.Generator().manual_seed(M + N + Kd)
    if grp:  # stored rows k live at (k // grp) * gstride + (k % grp) * ld: groups padded by 5 rows
        ng = (Kd + grp - 1) // grp
        Kd = ng * grp
        Ab = torch.randn(batch, ng, grp + 5, M, generator=g, dtype=torch.float64)
        Bb = torch.randn(batch, ng, grp + 5, N, generator=g, dtype=torch.float64)
        A = Ab[:, :, :grp].reshape(batch, Kd, M)
        B = Bb[:, :, :grp].reshape(batch, Kd, N)
        kw = dict(a_grp=grp, a_gs=(grp + 5) * M, b_grp=grp, b_gs=(grp + 5) * N, sa=ng * (grp + 5) * M,
                  sb=ng * (grp + 5) * N)
        Ad, Bd = Ab.float().to(cuda), Bb.float().to(cuda)
    else:
        A = torch.randn(batch, Kd, M, generator=g, dtype=torch.float64)
        B = torch.randn(batch, Kd, N, generator=g, dtype=torch.float64)
        kw = dict(sa=Kd * M, sb=Kd * N)
        Ad, Bd = A.float().to(cuda), B.float().to(cuda)
    C0 = torch.randn(batch, M, N, generator=g, dtype=torch.float64)
    b0 = torch.randn(batch, N, generator=g, dtype=torch.float64)
    Cd, bd = C0.float().to(cuda), b0.float().to(cuda)
    K.gemm(Ad, Bd, Cd, M, N, Kd, ta=True, batch=batch, sc=M * N, alpha=0.5, beta=1.0, bias_grad=bd, **kw)
    torch.cuda.synchronize()
    ref = 0.5 * A.transpose(1, 2) @ B + C0
    refb = 0.5 * B.sum(1) + b0
    scale = (A.abs().transpose(1, 2) @ B.abs()).max().item()
    assert (Cd.double().cpu() - ref).abs().max().item() <= 2e-6 * scale + 1e-5
    assert (bd.double().cpu() - refb).abs().max().item() <= 2e-6 * B.abs().sum(1).max().item() + 1e-5


@pytest.mark.parametrize("M,N,Kd", [(300, 64, 32), (300, 64, 64), (300, 64, 96), (300, 192, 64), (70, 40, 20),
                                     (300, 64, 2), (70, 24, 7)])
@pytest.mark.parametrize("beta,with_add", [(0.0, True), (0.7, False), (0.7, True)])
def test_gemm_epilogue_order_is_path_independent(cuda, M, N, Kd, beta, with_add):
    """Every GEMM path applies one epilogue order, (alpha acc + bias) + (beta C + addend): the rows kernels
    (whole-unit prefetch K <= 32 / N > 64, B-in-registers N <= 64 K = 64, plain K > 64), the tiled kernel (taken
    for op(A) = A^T) and its split-K reduce give the same bits.  Integer A and B make every accumulation exact in
    any order, so the epilogue is the only possible difference."""
    g = torch.Generator().manual_seed(M + N + Kd)
    A = torch.randint(-3, 4, (M, Kd), generator=g).float()
    B = torch.randint(-3, 4, (Kd, N), generator=g).float()
    C0 = torch.randn(M, N, generator=g)
    bias = torch.randn(N, generator=g)
    add = torch.randn(M, N, generator=g) if with_add else None
    outs = []
    for ta, split in ((False, 1), (True, 1), (True, 2)):
        Cd = C0.to(cuda).clone()
        Ad = (A.t().contiguous() if ta else A).to(cuda)
        K.gemm(Ad, B.to(cuda), Cd, M, N, Kd, ta=ta, bias=bias.to(cuda), addend=None if add is None else add.to(cuda),
               alpha=0.3, beta=beta, split_k=split)
        torch.cuda.synchronize()
        outs.append(Cd.cpu())
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[1], outs[2])
    ref = (0.3 * A.double() @ B.double() + bias.double()) + (beta * C0.double() + (0 if add is None else add.double()))
    assert (outs[0].double() - ref).abs().max().item() <= 1e-5 * (1 + ref.abs().max().item())


def test_gemm_row_grouping(cuda):
    """agent rows (first n of N per graph) as GEMM rows, in and out."""
    G, N, n, D, F = 5, 9, 3, 6, 4
    X = torch.randn(G, N, D, dtype=torch.float64)
    W = torch.randn(D, F, dtype=torch.float64)
    Y = torch.zeros(G, N, F, dtype=torch.float32, device=cuda)
    K.gemm(X.float().to(cuda), W.float().to(cuda), Y, G * n, F, D, lda=D, a_grp=n, a_gs=N * D, c_grp=n, c_gs=N * F)
    torch.cuda.synchronize()
    ref = X[:, :n] @ W
    assert (Y[:, :n].double().cpu() - ref).abs().max() < 1e-5
    assert Y[:, n:].abs().max() == 0


# ---- network fixtures ----------------------------------------------------------------------------
def _graphs(cuda, eid, n, obs, S, L, seed=0):
    env = make_env(eid, n, num_obs=obs, device=cuda)
    g = env.reset(key=seed, n_env=S)
    gs = []
    rng = np.random.default_rng(seed)
    for t in range(L):
        gs.append(g)
        a = torch.from_numpy(rng.uniform(-1, 1, (S, n, env.action_dim)).astype(np.float32)).to(cuda)
        g = env.step(g, a).graph
    stack = lambda f: torch.stack([getattr(x, f) for x in gs], 1).contiguous()  # noqa: E731
    nodes, edges, recv, send = stack("nodes"), stack("edges"), stack("receivers"), stack("senders")
    gb = GraphBatch(nodes.view(S * L, *nodes.shape[2:]), edges.view(S * L, *edges.shape[2:]),
                    recv.view(S * L, -1), send.view(S * L, -1), n, env.agent_candidates(cuda),
                    raw_cols=env.nonagent_feature_cols)
    host = dict(nodes=gb.nodes.cpu().numpy(), edges=gb.edges.cpu().numpy(), receivers=gb.receivers.cpu().numpy(),
                senders=gb.senders.cpu().numpy())
    return env, gb, host


CASES = [("LidarSpread", 8, 3), ("MPETarget", 3, 0), ("MPESpread", 3, 3), ("LidarBicycleTarget", 4, 2),
         ("LidarBicycleTarget", 8, 3)]  # BASELINE's bicycle config at its own n = 8, obs = 3
# 10-wide nodes and edges, 3-d actions: edge columns 4.. through edge_wsum / edge_da, agent-mode raw columns
OMNI = [("LidarOmniTarget", 3, 2), ("LidarOmniTarget", 8, 3)]
# BASELINE's dense-graph config: 72 candidate edges per agent (past the row-block kernels' 32)
DENSE = [("LidarSpread", 32, 8)]
# VMAS: 13 / 20-wide nodes (raw-row columns), agent-only graphs (3 candidate edges per agent)
VMAS = [("VMASWheel", 3, 0), ("VMASReverseTransport", 3, 0)]


def _nets_kw(env):
    return dict(edge_dim=env.edge_dim)


@pytest.mark.parametrize("eid,n,obs", CASES + OMNI + DENSE + VMAS)
def test_actor_eval_seq_fwd_bwd(cuda, eid, n, obs):
    S, L = 3, 4
    env, gb, host = _graphs(cuda, eid, n, obs, S, L)
    A = env.action_dim
    net = ActorNet(env.node_dim, n, cuda, seed=3, action_dim=A, **_nets_kw(env))
    rng = np.random.default_rng(1)
    actions = rng.uniform(-0.99, 0.99, (S * L * n, A)).astype(np.float32)
    actions[0, :2] = [0.9995, -0.9999]  # both boundary branches of the clipped log_prob
    eps = rng.standard_normal((n, A)).astype(np.float32)
    lp, ent, cache = net.eval_seq_fwd(gb, S, L, torch.from_numpy(actions).to(cuda), torch.from_numpy(eps).to(cuda))
    p = R.to_t(net.flax(), requires_grad=True)
    rlp, rent = R.actor_eval_seq(p, host, S, L, n, actions, eps)
    torch.cuda.synchronize()
    _close(lp.cpu().numpy(), rlp.detach().numpy().reshape(-1), what="log_pi")
    _close(ent.cpu().numpy(), rent.detach().numpy().reshape(-1), what="entropy")
    # gradients of an arbitrary scalar function of (log_pi, entropy)
    w1 = rng.standard_normal(S * L * n)
    w2 = rng.standard_normal(S * L * n)
    (rlp.reshape(-1) * torch.tensor(w1) + rent.reshape(-1) * torch.tensor(w2)).sum().backward()
    net.ps.zero_grad()
    net.eval_seq_bwd(cache, torch.tensor(w1, dtype=torch.float32, device=cuda),
                     torch.tensor(w2, dtype=torch.float32, device=cuda))
    torch.cuda.synchronize()
    net.ps.swap_views()
    g = net.flax()
    net.ps.swap_views()
    for path, a, b in _walk(g, R.grads(p)):
        _grad_close(a, b, "actor grad " + path)


@pytest.mark.parametrize("eid,n,obs", CASES[:2] + CASES[4:] + OMNI[:1] + VMAS)
def test_vl_seq_fwd_bwd(cuda, eid, n, obs):
    S, L = 3, 5
    env, gb, host = _graphs(cuda, eid, n, obs, S, L, seed=4)
    net = VlNet(env.node_dim, n, cuda, seed=5, **_nets_kw(env))
    v, _, cache = net.seq_fwd(gb, S, L)
    p = R.to_t(net.flax(), requires_grad=True)
    rv = R.vl_seq(p, host, S, L, n)
    torch.cuda.synchronize()
    _close(v.cpu().numpy(), rv.detach().numpy(), what="Vl")
    w = np.random.default_rng(2).standard_normal((S, L))
    (rv * torch.tensor(w)).sum().backward()
    net.ps.zero_grad()
    net.seq_bwd(cache, torch.tensor(w, dtype=torch.float32, device=cuda))
    torch.cuda.synchronize()
    net.ps.swap_views()
    g = net.flax()
    net.ps.swap_views()
    for path, a, b in _walk(g, R.grads(p)):
        _grad_close(a, b, "Vl grad " + path)


@pytest.mark.parametrize("eid,n,obs", CASES[:3] + CASES[4:] + OMNI[:1] + DENSE + VMAS)
def test_vh_fwd_bwd(cuda, eid, n, obs):
    S, L = 2, 3
    env, gb, host = _graphs(cuda, eid, n, obs, S, L, seed=6)
    net = VhNet(env.node_dim, n, 2, cuda, seed=7, **_nets_kw(env))
    h = np.random.default_rng(3).standard_normal((S * L * n, 64)).astype(np.float32) * 0.5
    out, cache = net.fwd(gb, torch.from_numpy(h).to(cuda))
    p = R.to_t(net.flax(), requires_grad=True)
    rout = R.vh(p, host, h.reshape(S * L, n, 64), n)
    torch.cuda.synchronize()
    _close(out.cpu().numpy(), rout.detach().numpy().reshape(-1, 2), what="Vh")
    w = np.random.default_rng(4).standard_normal(rout.shape)
    (rout * torch.tensor(w)).sum().backward()
    net.ps.zero_grad()
    net.bwd(cache, torch.tensor(w.reshape(-1, 2), dtype=torch.float32, device=cuda))
    torch.cuda.synchronize()
    net.ps.swap_views()
    g = net.flax()
    net.ps.swap_views()
    for path, a, b in _walk(g, R.grads(p)):
        _grad_close(a, b, "Vh grad " + path)


@pytest.mark.parametrize("fused", ["1", "0"])
@pytest.mark.parametrize("layers", [2, 1])
@pytest.mark.parametrize("eid,n,obs", CASES + OMNI[:1] + DENSE + VMAS)
def test_actor_act_step(cuda, monkeypatch, eid, n, obs, layers, fused):
    """ActorNet.act (PPOPolicy.get_action / sample_action, policy.py:191-212) for one graph batch with
    non-zero carries, through the fused dgppo_policy_step kernel ("1") and the unfused layer chain
    ("0"): carry, action (tanh of mean, or of mean + std * noise) and log_pi against float64."""
    monkeypatch.setenv("DGPPO_FUSED_POLICY", fused)
    S, L = 5, 3  # 15 graphs: partial last row group in the fused kernel for every n
    env, gb, host = _graphs(cuda, eid, n, obs, S, L, seed=2)
    A = env.action_dim
    net = ActorNet(env.node_dim, n, cuda, seed=5, gnn_layers=layers, action_dim=A, **_nets_kw(env))
    rows = S * L * n
    rng = np.random.default_rng(4)
    h = torch.from_numpy(rng.standard_normal((rows, 64)).astype(np.float32) * 0.5).to(cuda)
    noise = torch.from_numpy(rng.standard_normal((rows, A)).astype(np.float32)).to(cuda)
    p = R.to_t(net.flax())
    h2_ref = R.actor_carry(p, host, h.cpu().double().reshape(S * L, n, 64), n)
    mu, sd = R.policy_dist(p, h2_ref)
    try:  # the same oracle in float32: the noise floor of an fp32 evaluation (module docstring)
        R.T64 = torch.float32
        p32 = R.to_t(net.flax())
        h2_32 = R.actor_carry(p32, host, h.cpu().float().reshape(S * L, n, 64), n)
        mu32, sd32 = R.policy_dist(p32, h2_32)
    finally:
        R.T64 = torch.float64
    for mode in (0, 1):
        a, lp, h2 = net.act(gb, h, mode, noise=noise if mode else None)
        torch.cuda.synchronize()
        _close(h2.cpu().numpy(), h2_ref.numpy().reshape(rows, 64), what=f"carry mode {mode}")
        pre = mu + sd * noise.cpu().double().reshape(S * L, n, A) if mode else mu
        a_ref = torch.tanh(pre)
        _close(a.cpu().numpy(), a_ref.numpy().reshape(rows, A), what=f"action mode {mode}")
        a_host = a.cpu().double().reshape(S * L, n, A)
        lp_ref = R.tanh_normal_log_prob(a_host, mu, sd).numpy().reshape(rows)
        lp_32 = R.tanh_normal_log_prob(a_host.float(), mu32.double(), sd32.double()).numpy().reshape(rows)
        # log pi of the GPU's own fp32 action: 1e-5 (1 + |ref|) plus 8x the float32-oracle floor (the
        # atanh / log(1 - a^2) terms amplify the mean / std rounding near |a| -> 1)
        err = np.abs(lp.cpu().numpy() - lp_ref)
        floor = np.abs(lp_32 - lp_ref)
        assert (err - 1e-5 * (1 + np.abs(lp_ref)) - 8 * floor).max() <= 0, \
            f"log_pi mode {mode}: max abs err {err.max():.3e}, fp32 floor {floor.max():.3e}"


# ---- known-answer test on the attention kernels ----------------------------------
@pytest.mark.parametrize("eid,n,obs,layers", [("LidarSpread", 8, 3, 2), ("MPESpread", 3, 3, 2), ("LidarSpread", 32, 8, 2),
                                              ("LidarSpread", 8, 3, 3)])
def test_attention_uniform_logits_give_inverse_in_degree(cuda, eid, n, obs, layers):
    """Wq = 0, bq = 0 makes every logit q.k/sqrt(F) zero, so jraph.segment_softmax gives each of a
    receiver's in-edges weight exactly 1 / in-degree (masked candidates 0), in every layer (the
    first reads raw sender rows, the second is the agent-mode kernel, a third reads materialised rows)."""
    S, L = 2, 3
    env, gb, host = _graphs(cuda, eid, n, obs, S, L, seed=9)
    net = ActorNet(env.node_dim, n, cuda, seed=1, gnn_layers=layers, action_dim=env.action_dim, **_nets_kw(env))
    for layer in net.gnn.layers:
        layer.v("Wq").zero_()
        layer.v("bq").zero_()
    _, (caches, _) = net.gnn.fwd(gb)
    torch.cuda.synchronize()
    recv = host["receivers"]
    deg = np.stack([(recv == i).sum(1) for i in range(n)], 1).reshape(-1)  # (G*n,) in-degree of agent rows
    valid = gb.sidx.cpu().numpy() >= 0  # (G*n, C)
    assert (valid.sum(1) == deg).all()
    for li, c in enumerate(caches):
        attn = c[4].cpu().numpy()  # (G*n, H, C)
        want = np.where(valid[:, None, :], 1.0 / np.maximum(deg, 1)[:, None, None], 0.0)
        want = np.broadcast_to(want, attn.shape)
        np.testing.assert_allclose(attn, want, rtol=2e-7, atol=0, err_msg=f"layer {li}")


@pytest.mark.parametrize("S,L", [(3, 128), (2, 200)])
def test_vl_long_scan_matches_oracle(cuda, S, L):
    """The update's prepass scans Vl over a whole episode (L = T = 128, scan_Vl informarl.py:281-293):
    every step of a long GRU scan against the float64 oracle."""
    env, gb, host = _graphs(cuda, "LidarSpread", 4, 2, S, L, seed=11)
    net = VlNet(env.node_dim, 4, cuda, seed=12, **_nets_kw(env))
    v, hT, _ = net.seq_fwd(gb, S, L, keep_cache=False)
    p = R.to_t(net.flax())
    rv, rh = R.vl_seq(p, host, S, L, 4, return_h=True)
    torch.cuda.synchronize()
    _close(v.cpu().numpy(), rv.detach().numpy(), what="Vl over a long scan")
    _close(hT.cpu().numpy(), rh.detach().numpy(), what="final carry")


# GNN stacks deeper than the reference's defaults (--actor-gnn-layers / --Vl-gnn-layers / --Vh-gnn-layers > 2,
# train.py): layers past the second read materialised node rows (agents: the previous layer's outputs; every other
# node: its lifted Dense_4 + ReLU chain, nn/layers.py GNN.fwd) and their backward returns every sender's gradient
DEEP = [("LidarSpread", 8, 3, 3), ("LidarOmniTarget", 3, 2, 3), ("MPESpread", 3, 3, 4)]


@pytest.mark.parametrize("eid,n,obs,layers", DEEP)
def test_deep_gnn_nets_fwd_bwd(cuda, eid, n, obs, layers):
    S, L = 2, 3
    env, gb, host = _graphs(cuda, eid, n, obs, S, L, seed=8)
    A = env.action_dim
    rng = np.random.default_rng(11)
    # actor: eval_action over the sequences (log pi, entropy and every gradient)
    net = ActorNet(env.node_dim, n, cuda, seed=9, gnn_layers=layers, action_dim=A, **_nets_kw(env))
    assert len(net.gnn.layers) == layers and net._fused_args(gb) is None
    actions = rng.uniform(-0.99, 0.99, (S * L * n, A)).astype(np.float32)
    eps = rng.standard_normal((n, A)).astype(np.float32)
    lp, ent, cache = net.eval_seq_fwd(gb, S, L, torch.from_numpy(actions).to(cuda), torch.from_numpy(eps).to(cuda))
    p = R.to_t(net.flax(), requires_grad=True)
    rlp, rent = R.actor_eval_seq(p, host, S, L, n, actions, eps)
    torch.cuda.synchronize()
    _close(lp.cpu().numpy(), rlp.detach().numpy().reshape(-1), what="log_pi")
    _close(ent.cpu().numpy(), rent.detach().numpy().reshape(-1), what="entropy")
    w1, w2 = rng.standard_normal(S * L * n), rng.standard_normal(S * L * n)
    (rlp.reshape(-1) * torch.tensor(w1) + rent.reshape(-1) * torch.tensor(w2)).sum().backward()
    net.ps.zero_grad()
    net.eval_seq_bwd(cache, torch.tensor(w1, dtype=torch.float32, device=cuda),
                     torch.tensor(w2, dtype=torch.float32, device=cuda))
    torch.cuda.synchronize()
    net.ps.swap_views()
    g = net.flax()
    net.ps.swap_views()
    for path, a, b in _walk(g, R.grads(p)):
        _grad_close(a, b, f"deep actor grad {path}")
    # one policy step (the rollout's unfused path) with non-zero carries
    h = torch.from_numpy(rng.standard_normal((S * L * n, 64)).astype(np.float32) * 0.5).to(cuda)
    _, _, h2 = net.act(gb, h, 0)
    h2_ref = R.actor_carry(R.to_t(net.flax()), host, h.cpu().double().reshape(S * L, n, 64), n)
    torch.cuda.synchronize()
    _close(h2.cpu().numpy(), h2_ref.numpy().reshape(-1, 64), what="carry")
    # Vl: values and gradients over the sequences
    vl = VlNet(env.node_dim, n, cuda, seed=10, gnn_layers=layers, **_nets_kw(env))
    v, _, vc = vl.seq_fwd(gb, S, L)
    pv = R.to_t(vl.flax(), requires_grad=True)
    rv = R.vl_seq(pv, host, S, L, n)
    torch.cuda.synchronize()
    _close(v.cpu().numpy(), rv.detach().numpy(), what="Vl")
    w = rng.standard_normal((S, L))
    (rv * torch.tensor(w)).sum().backward()
    vl.ps.zero_grad()
    vl.seq_bwd(vc, torch.tensor(w, dtype=torch.float32, device=cuda))
    torch.cuda.synchronize()
    vl.ps.swap_views()
    g = vl.flax()
    vl.ps.swap_views()
    for path, a, b in _walk(g, R.grads(pv)):
        _grad_close(a, b, f"deep Vl grad {path}")


# the reference CLI's RNN options (--rnn-layers, --use-lstm, --no-rnn; dgppo/nn/rnn.py:10-30): RNN(GRUCell |
# LSTMCell, layers) with (layers, carries, 64) carries per agent, or no RNN (features pass through)
RNNS = [("gru", 2), ("lstm", 1), ("lstm", 2), ("none", 1)]


@pytest.mark.parametrize("kind,layers", RNNS)
def test_rnn_options_nets_fwd_bwd(cuda, kind, layers):
    eid, n, obs = "LidarSpread", 4, 2
    S, L = 2, 4
    env, gb, host = _graphs(cuda, eid, n, obs, S, L, seed=12)
    A, rows = env.action_dim, S * L * n
    rng = np.random.default_rng(13)
    rk = dict(rnn=kind, rnn_layers=layers)
    net = ActorNet(env.node_dim, n, cuda, seed=14, action_dim=A, **_nets_kw(env), **rk)
    W = net.carry_width
    assert W == (128 if kind == "lstm" else 64) * layers and net._fused_args(gb) is None
    actions = rng.uniform(-0.99, 0.99, (rows, A)).astype(np.float32)
    eps = rng.standard_normal((n, A)).astype(np.float32)
    lp, ent, cache = net.eval_seq_fwd(gb, S, L, torch.from_numpy(actions).to(cuda), torch.from_numpy(eps).to(cuda))
    p = R.to_t(net.flax(), requires_grad=True)
    rlp, rent = R.actor_eval_seq(p, host, S, L, n, actions, eps)
    torch.cuda.synchronize()
    _close(lp.cpu().numpy(), rlp.detach().numpy().reshape(-1), what="log_pi")
    _close(ent.cpu().numpy(), rent.detach().numpy().reshape(-1), what="entropy")
    w1, w2 = rng.standard_normal(rows), rng.standard_normal(rows)
    (rlp.reshape(-1) * torch.tensor(w1) + rent.reshape(-1) * torch.tensor(w2)).sum().backward()
    net.ps.zero_grad()
    net.eval_seq_bwd(cache, torch.tensor(w1, dtype=torch.float32, device=cuda),
                     torch.tensor(w2, dtype=torch.float32, device=cuda))
    torch.cuda.synchronize()
    net.ps.swap_views()
    g = net.flax()
    net.ps.swap_views()
    for path, a, b in _walk(g, R.grads(p)):
        _grad_close(a, b, f"{kind}{layers} actor grad {path}")
    # one policy step from non-zero carries (the rollout's act): the new carries and the action
    h = rng.standard_normal((rows, W)).astype(np.float32) * 0.5
    a, _, h2 = net.act(gb, torch.from_numpy(h).to(cuda), 0)
    pq = R.to_t(net.flax())
    hh = torch.as_tensor(h, dtype=torch.float64).reshape(S * L, n, W)
    h2_ref = R.actor_carry(pq, host, hh, n)
    feat, _ = R.rnn(pq["gru"], hh, R.mlp_head(R.gnn(pq["gnn"], host, n), pq["head"]))
    mu, _ = R.policy_dist(pq, feat)
    torch.cuda.synchronize()
    _close(h2.cpu().numpy(), h2_ref.numpy().reshape(rows, W), what="carry")
    _close(a.cpu().numpy(), torch.tanh(mu).numpy().reshape(rows, A), what="action")
    # Vl from given initial carries: values, final carries, gradients
    vl = VlNet(env.node_dim, n, cuda, seed=15, **_nets_kw(env), **rk)
    h0 = rng.standard_normal((S, W)).astype(np.float32) * 0.5
    v, hT, vc = vl.seq_fwd(gb, S, L, h0=torch.from_numpy(h0).to(cuda))
    pv = R.to_t(vl.flax(), requires_grad=True)
    rv, rhT = R.vl_seq(pv, host, S, L, n, h0=h0.astype(np.float64), return_h=True)
    torch.cuda.synchronize()
    _close(v.cpu().numpy(), rv.detach().numpy(), what="Vl")
    _close(hT.cpu().numpy(), rhT.detach().numpy(), what="Vl final carry")
    w = rng.standard_normal((S, L))
    (rv * torch.tensor(w)).sum().backward()
    vl.ps.zero_grad()
    vl.seq_bwd(vc, torch.tensor(w, dtype=torch.float32, device=cuda))
    torch.cuda.synchronize()
    vl.ps.swap_views()
    g = vl.flax()
    vl.ps.swap_views()
    for path, a, b in _walk(g, R.grads(pv)):
        _grad_close(a, b, f"{kind}{layers} Vl grad {path}")
    # Vh on the actor's carries
    vh = VhNet(env.node_dim, n, 2, cuda, seed=16, **_nets_kw(env), **rk)
    out, hc = vh.fwd(gb, torch.from_numpy(h).to(cuda))
    ph = R.to_t(vh.flax(), requires_grad=True)
    rout = R.vh(ph, host, hh, n)
    torch.cuda.synchronize()
    _close(out.cpu().numpy(), rout.detach().numpy().reshape(-1, 2), what="Vh")
    wv = rng.standard_normal(rout.shape)
    (rout * torch.tensor(wv)).sum().backward()
    vh.ps.zero_grad()
    vh.bwd(hc, torch.tensor(wv.reshape(-1, 2), dtype=torch.float32, device=cuda))
    torch.cuda.synchronize()
    vh.ps.swap_views()
    g = vh.flax()
    vh.ps.swap_views()
    for path, a, b in _walk(g, R.grads(ph)):
        _grad_close(a, b, f"{kind}{layers} Vh grad {path}")


def test_graph_forward_on_the_fly_rows_bit_identical(cuda):
    """ABI 10 dgppo_gnn_set_graph_otf: the graph-form forward of the dense n = 32 graphs with each receiver's own hit
    rows computed on the fly (LDS holds only the agent and goal rows) gives the same bits as staging every row --
    values, and the gradients of the backward that reads the forward's attention weights and xcat rows."""
    from dgppo_fov_amd import _lib
    S, L = 2, 3
    env, gb, _ = _graphs(cuda, "LidarSpread", 32, 8, S, L, seed=5)
    lib = _lib.load()
    res = []
    try:
        for otf in (1, 0):
            assert lib.dgppo_gnn_set_graph_otf(otf) == 0
            net = VlNet(env.node_dim, 32, cuda, seed=9, **_nets_kw(env))
            v, hT, cache = net.seq_fwd(gb, S, L)
            net.ps.zero_grad()
            net.seq_bwd(cache, torch.linspace(-1.0, 1.0, S * L, device=cuda).view(S, L))
            torch.cuda.synchronize()
            res.append((v.cpu(), hT.cpu(), net.ps.grad.cpu().clone()))
    finally:
        lib.dgppo_gnn_set_graph_otf(1)
    for a, b, what in zip(res[0], res[1], ("values", "carries", "gradients")):
        assert torch.equal(a, b), what
    assert res[0][2].abs().max() > 0

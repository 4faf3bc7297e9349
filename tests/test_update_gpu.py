"""GPU parity for the DGPPO update (hot path 2 end to end): Dec-OCP GAE, merged DGPPO advantage,
global-norm clip + apply_if_finite Adam, and one full `DGPPO.update` (prepass Vl/Vh on both rollouts,
targets, advantages, Vl/Vh/policy losses and gradients, Adam) against the float64 restatement in
oracle/nets.py + oracle/nets_t.py (dgppo.py:136-321, informarl.py:357-457, algo/utils.py:11-79).

Tolerances (fp32 kernels vs float64), north_star's 1e-5: every value, target and advantage satisfies
|gpu - ref64| <= 1e-5 (1 + |ref64|) + 8 |ref32 - ref64|, where ref32 is the SAME oracle evaluated in
float32 (the noise floor any fp32 evaluation of these networks has: ReLU gates and softmax weights
decided by rounding); advantages are compared where every CBF-derivative component is farther than
1e-3 from the is_safe threshold (a sign decided by fp32 noise is not a parity failure); gradients
within 2e-5 of the largest reference entry + 8x the same float32 floor; Adam results within 1e-6
absolute (lr-sized steps).  Known-answer tests: Adam one step on a quadratic.
"""
import numpy as np
import pytest
import torch

from dgppo_fov_amd.algo import make_algo
from dgppo_fov_amd.algo.dgppo import DGPPO
from dgppo_fov_amd.env import make_env
from dgppo_fov_amd.nn import kernels as K
from oracle import nets as O
from oracle import nets_t as R

pytestmark = pytest.mark.gpu


def _close(a, b, tol, what):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    err = (np.abs(a - b) - tol * (1 + np.abs(b))).max()
    assert err <= 0, f"{what}: max abs err {np.abs(a - b).max():.3e}"


def _close_floor(a, r64, r32, what, tol=1e-5, floor=None):
    """|a - r64| <= tol (1 + |r64|) + 8 floor, floor = |r32 - r64| elementwise unless given (see module
    docstring)."""
    a, r64, r32 = (np.asarray(x, np.float64) for x in (a, r64, r32))
    err = np.abs(a - r64)
    floor = np.abs(r32 - r64) if floor is None else np.asarray(floor, np.float64)
    excess = (err - tol * (1 + np.abs(r64)) - 8 * floor).max()
    assert excess <= 0, (f"{what}: max abs err {err.max():.3e}, max rel err {(err / (1 + np.abs(r64))).max():.3e}, "
                         f"fp32 floor {floor.max():.3e}")


def _walk(a, b, path=""):
    if isinstance(a, dict):
        for k in a:
            yield from _walk(a[k], b[k], f"{path}/{k}")
    elif isinstance(a, list):
        for i, (x, y) in enumerate(zip(a, b)):
            yield from _walk(x, y, f"{path}[{i}]")
    else:
        yield path, a, b


# ---- GAE -------------------------------------------------------------------------------------
@pytest.mark.parametrize("B,T,n,nh", [(3, 1, 1, 1), (2, 32, 3, 2), (2, 128, 8, 2), (1, 255, 16, 2), (1, 128, 32, 2), (2, 40, 1, 1)])
def test_gae_matches_oracle(cuda, B, T, n, nh):
    rng = np.random.default_rng(T + n)
    hs = rng.standard_normal((B, T, n, nh)).astype(np.float32)
    l = rng.standard_normal((B, T)).astype(np.float32)
    Vh = rng.standard_normal((B, T + 1, n, nh)).astype(np.float32)
    Vl = rng.standard_normal((B, T + 1)).astype(np.float32)
    Qh = torch.empty((B, T, n, nh), device=cuda)
    Ql = torch.empty((B, T), device=cuda)
    d = lambda x: torch.from_numpy(x).to(cuda)  # noqa: E731
    K.gae(d(hs), d(l), d(Vh), d(Vl), Qh, Ql, 0.99, 0.95)
    torch.cuda.synchronize()
    for b in range(B):
        qh, ql = O.compute_dec_ocp_gae(hs[b].astype(np.float64), l[b].astype(np.float64), Vh[b].astype(np.float64),
                                       Vl[b].astype(np.float64), 0.99, 0.95)
        _close(Qh[b].cpu().numpy(), qh, 2e-5, f"Qh[{b}]")
        _close(Ql[b].cpu().numpy(), ql, 2e-5, f"Ql[{b}]")


# ---- DGPPO advantage ---------------------------------------------------------------------------
def test_dgppo_advantages_match_oracle(cuda):
    B, T, n, nh = 3, 64, 4, 2
    rng = np.random.default_rng(0)
    Ql = rng.standard_normal((B, T)).astype(np.float32)
    Vl = rng.standard_normal((B, T + 1)).astype(np.float32)
    Vh = (rng.standard_normal((B, T + 1, n, nh)) * 0.05).astype(np.float32)
    d = lambda x: torch.from_numpy(x).to(cuda)  # noqa: E731
    A = torch.empty((B, T, n), device=cuda)
    cnt = torch.empty(B, device=cuda)
    dt, alpha, eps, w = 0.03, 10.0, 1e-2, 2.0
    K.dgppo_advantages(d(Ql), d(Vl), d(Vh), A, cnt, dt, alpha, eps, w)
    torch.cuda.synchronize()
    Vh64 = Vh.astype(np.float64)
    Al = Ql - Vl[:, :T].astype(np.float64)
    Al = (Al - Al.mean(1, keepdims=True)) / (Al.std(1, keepdims=True) + 1e-8)
    deriv = (Vh64[:, 1:] - Vh64[:, :T]) / dt + alpha * Vh64[:, :T]
    safe = (deriv <= 0).min(-1)
    ref = -(np.where(safe, Al[..., None], 0) + np.maximum(deriv + eps, 0).max(-1) * w)
    robust = np.abs(deriv).min(-1) > 1e-3
    _close(A.cpu().numpy()[robust], ref[robust], 2e-5, "A")
    assert abs(cnt.sum().item() - safe.sum()) <= (~robust).sum()


# ---- clip + apply_if_finite Adam ------------------------------------------------------------------
@pytest.mark.parametrize("scale", [1e-3, 10.0])
def test_adam_clip_matches_optax_restatement(cuda, scale):
    rng = np.random.default_rng(5)
    n = 70_001
    p = rng.standard_normal(n).astype(np.float32)
    m = (rng.standard_normal(n) * 1e-3).astype(np.float32)
    v = (rng.random(n) * 1e-4).astype(np.float32)
    g = (rng.standard_normal(n) * scale).astype(np.float32)
    d = lambda x: torch.from_numpy(x.copy()).to(cuda)  # noqa: E731
    P, M, V, G = d(p), d(m), d(v), d(g)
    st = torch.tensor([0.0, 0.0, 4.0], device=cuda)
    K.grad_norm(G, st)
    K.adam(P, G, M, V, st, 1e-3, max_norm=2.0)
    torch.cuda.synchronize()
    (gc,), gn = O.clip_by_global_norm_ref([g], 2.0)
    (rp,), (rm,), (rv,) = O.adam_step([p.astype(np.float64)], [gc], [m.astype(np.float64)], [v.astype(np.float64)],
                                      4, 1e-3)
    assert abs(st[0].item() - gn) <= 1e-5 * gn
    assert st[1].item() == 0 and st[2].item() == 5
    assert np.abs(P.cpu().numpy() - rp).max() <= 1e-6
    _close(M.cpu().numpy(), rm, 1e-6, "m")
    _close(V.cpu().numpy(), rv, 1e-6, "v")


def test_adam_one_step_on_quadratic_kat(cuda):
    """Known answer: f(p) = 0.5 c p^2, g = c p, clipped to global norm 2, then the
    first optax adam step moves every coordinate by lr * g / (|g| + eps) (m_hat = g, v_hat = g^2)."""
    c, lr = 3.0, 1e-3
    p0 = np.array([2.0, -0.5, 1e-9, 0.0, 0.25], np.float32)
    g = (c * p0.astype(np.float64))
    gn = np.sqrt((g * g).sum())
    gc = g * 2.0 / max(2.0, gn)
    want = p0.astype(np.float64) - lr * gc / (np.abs(gc) + 1e-8)
    P = torch.from_numpy(p0.copy()).to(cuda)
    G = torch.from_numpy(g.astype(np.float32)).to(cuda)
    M, V = torch.zeros_like(P), torch.zeros_like(P)
    st = torch.zeros(3, device=cuda)
    K.grad_norm(G, st)
    K.adam(P, G, M, V, st, lr, max_norm=2.0)
    torch.cuda.synchronize()
    assert abs(st[0].item() - gn) <= 1e-6 * gn and st[2].item() == 1
    np.testing.assert_allclose(P.cpu().numpy(), want, rtol=0, atol=2e-7)
    np.testing.assert_allclose(M.cpu().numpy(), 0.1 * gc, rtol=1e-6, atol=1e-12)
    np.testing.assert_allclose(V.cpu().numpy(), 0.001 * gc * gc, rtol=1e-6, atol=1e-15)


def test_adam_skips_nonfinite_update(cuda):
    g = torch.ones(1000, device=cuda)
    g[17] = float("nan")
    p = torch.randn(1000, device=cuda)
    p0 = p.clone()
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    st = torch.zeros(3, device=cuda)
    K.grad_norm(g, st)
    K.adam(p, g, m, v, st, 1e-3)
    torch.cuda.synchronize()
    assert st[1].item() > 0 and st[2].item() == 0
    assert torch.equal(p, p0) and m.abs().max() == 0 and v.abs().max() == 0


# ---- one full DGPPO.update ---------------------------------------------------------------------
def _host(r, n):
    B, T = r.rewards.shape
    f = lambda G, sl: {k: getattr(G, k)[sl].cpu().numpy() for k in ("nodes", "edges", "receivers", "senders")}  # noqa
    return dict(graph=f(r.graph, slice(None)), last=f(r.next_graph, (slice(None), -1)),
                rewards=r.rewards.cpu().numpy(), costs=r.costs.cpu().numpy(),
                rnn=DGPPO._rows(r.rnn_states).reshape(B, T, n, -1).cpu().numpy(), actions=r.actions.cpu().numpy(),
                log_pis=None if r.log_pis is None else r.log_pis.cpu().numpy())


def _net_trees(algo, grad=False):
    out = []
    for net in (algo.actor, algo.Vl, algo.Vh):
        if grad:
            net.ps.swap_views()
        out.append(net.flax())
        if grad:
            net.ps.swap_views()
    return out


@pytest.mark.parametrize("eid,n,obs,B", [("LidarSpread", 3, 2, 4), ("MPESpread", 3, 3, 4), ("LidarBicycleTarget", 2, 1, 4),
                                         ("LidarOmniTarget", 3, 2, 4), ("LidarSpread", 32, 8, 4),
                                         # the BASELINE bench shape and the bicycle config at n = 8, obs = 3
                                         ("LidarSpread", 8, 3, 8), ("LidarBicycleTarget", 8, 3, 8)])
def test_dgppo_update_matches_oracle(cuda, eid, n, obs, B):
    _update_parity(cuda, eid, n, obs, B)


# the reference CLI's RNN options (--rnn-layers, --use-lstm, --no-rnn): RNN(GRUCell | LSTMCell, layers) or none
@pytest.mark.parametrize("rk", [dict(rnn_layers=2), dict(use_lstm=True), dict(use_lstm=True, rnn_layers=2),
                                dict(use_rnn=False)], ids=["gru2", "lstm1", "lstm2", "no_rnn"])
def test_dgppo_update_rnn_options_match_oracle(cuda, rk):
    _update_parity(cuda, "LidarSpread", 3, 2, 4, **rk)


def _update_parity(cuda, eid, n, obs, B, **rk):
    T, L = 32, 16
    env = make_env(eid, n, num_obs=obs, max_step=T, device=cuda)
    algo = make_algo("dgppo", env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                     action_dim=env.action_dim, n_agents=n, batch_size=B * T, rnn_step=L, train_steps=100,
                     seed=1, device=cuda, **rk)
    roll = algo.collect(algo.params, 7, n_env=B)
    lay, car = rk.get("rnn_layers", 1), 2 if rk.get("use_lstm") and rk.get("use_rnn", True) else 1
    assert roll.rnn_states.shape == (B, T, lay, n, car, 64)
    pa, pl, ph = _net_trees(algo)
    algo.trace = {}
    info = algo.update(roll, 60)  # past 50% of train_steps: cbf weight doubled
    torch.cuda.synchronize()
    tr = algo.trace
    hr, hd = _host(roll, n), _host(tr["det"], n)
    cw = algo.cbf_weight_at(60)
    assert cw == 2.0
    refs = {}
    try:
        for dt in (torch.float64, torch.float32):
            R.T64 = dt
            refs[dt] = R.dgppo_prepass(R.to_t(pa), R.to_t(pl), R.to_t(ph), hr, hd, n, env.dt, algo.gamma,
                                       algo.gae_lambda, algo.alpha, algo.cbf_eps, cw)
    finally:
        R.T64 = torch.float64
    ref, ref32 = refs[torch.float64], refs[torch.float32]
    for k in ("Vl", "Vh", "Vh_det", "Ql", "Qh", "Qh_det"):
        _close_floor(tr[k].cpu().numpy(), ref[k], ref32[k], k)
    robust = np.abs(ref["deriv"]).min(-1) > 1e-3
    assert robust.mean() > 0.5
    # A = (Al - mean_t Al) / std_t Al couples all T steps of an env: its fp32 floor is the env's largest
    env_floor = np.broadcast_to(np.abs(ref32["A"] - ref["A"]).max(axis=(1, 2), keepdims=True), ref["A"].shape)
    _close_floor(tr["A"].cpu().numpy()[robust], ref["A"][robust], ref32["A"][robust], "A", floor=env_floor[robust])
    total = B * T * n
    assert abs(info["eval/safe_data"] - ref["safe_data"]) <= (~robust).sum() / total + 1e-6

    # gradients of the single minibatch, oracle fed the GPU's own targets / advantages; the same
    # oracle evaluated in float32 gives the noise floor of an fp32 evaluation (ReLU gates and
    # softmax weights decided by rounding make some tensors differ from float64 by far more than
    # 2e-5 relative, identically for any fp32 implementation)
    (mb,) = tr["mb"]
    algo.grad_flat.copy_(mb["grad"])
    gpu = _net_trees(algo, grad=True)
    envs = np.asarray(mb["envs"])
    refs = {}
    try:
        for dt in (torch.float64, torch.float32):
            R.T64 = dt
            ts = [R.to_t(x, requires_grad=True) for x in (pa, pl, ph)]
            losses = R.dgppo_minibatch_grads(*ts, hr, hd, envs, tr["Ql"].double().cpu().numpy(),
                                             tr["Qh_det"].double().cpu().numpy(), tr["A"].double().cpu().numpy(),
                                             n, L, algo.entropy_eps.cpu().numpy(), algo.clip_eps, algo.coef_ent)
            refs[dt] = ([R.grads(t) for t in ts], losses)
    finally:
        R.T64 = torch.float64
    losses = refs[torch.float64][1]
    _close(info["Vl/loss"], losses["Vl_loss"], 1e-5, "Vl loss")
    _close(info["Vh/loss_Vh"], losses["Vh_loss"], 1e-5, "Vh loss")
    _close(info["policy/loss"], losses["policy_loss"], 1e-5, "policy loss")
    _close(info["policy/entropy"], losses["entropy"], 1e-5, "entropy")
    for tag, g, r64, r32 in zip(("actor", "Vl", "Vh"), gpu, refs[torch.float64][0], refs[torch.float32][0]):
        for (path, a, b), (_, c, _) in zip(_walk(g, r64), _walk(r32, r64)):
            b = np.asarray(b, np.float64)
            err = np.abs(np.asarray(a, np.float64) - b).max()
            floor = np.abs(np.asarray(c, np.float64) - b).max()
            assert err <= 2e-5 * np.abs(b).max() + 1e-6 + 8 * floor, f"{tag} grad {path}: {err:.3e} (fp32 floor {floor:.3e})"

    # clip + Adam on exactly those gradients
    off = 0
    for name, net in (("Vl", algo.Vl), ("Vh", algo.Vh), ("policy", algo.actor)):
        sz = net.ps.size
        g = mb["grad"][off:off + sz].double().cpu().numpy()
        off += sz
        (gc,), gn = O.clip_by_global_norm_ref([g], algo.max_grad_norm)
        key = {"Vl": "Vl/grad_norm", "Vh": "Vh/grad_Vh_norm", "policy": "policy/grad_norm"}[name]
        assert abs(info[key] - gn) <= 1e-5 * gn
        (rp,), _, _ = O.adam_step([mb["before"][name].double().cpu().numpy()], [gc], [np.zeros(sz)], [np.zeros(sz)],
                                  0, algo.opt[name].lr)
        assert np.abs(net.ps.flat.double().cpu().numpy() - rp).max() <= 1e-6, name


def test_checkpoint_round_trip(cuda, tmp_path):
    env = make_env("MPETarget", 3, num_obs=0, max_step=16, device=cuda)
    kw = dict(env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
              action_dim=env.action_dim, n_agents=3, batch_size=64, rnn_step=16, device=cuda)
    a = make_algo("dgppo", seed=3, **kw)
    a.update(a.collect(a.params, 1, n_env=8), 0)
    a.save(str(tmp_path), 7)
    b = make_algo("dgppo", seed=4, **kw)
    b.load(str(tmp_path), 7)
    for k in ("policy", "Vl", "Vh"):
        assert torch.equal(a.params[k], b.params[k])
    for k in a.opt:
        assert torch.equal(a.opt[k].m, b.opt[k].m) and torch.equal(a.opt[k].state, b.opt[k].state)
    ra, rb = a.collect(a.params, 5, n_env=8), b.collect(b.params, 5, n_env=8)
    assert torch.equal(ra.actions, rb.actions)


def test_update_graph_replay_matches_eager(cuda, monkeypatch):
    """The minibatch step replayed from its captured hipGraph (DGPPO_UPDATE_GRAPH=1: minibatch 0 eager +
    capture, the rest replays; the next update replays every minibatch) gives bit-identical
    parameters, Adam state and info to the eager step, over two updates."""
    eid, n, obs, B, T = "LidarSpread", 3, 2, 8, 32

    def run(flag):
        monkeypatch.setenv("DGPPO_UPDATE_GRAPH", flag)
        env = make_env(eid, n, num_obs=obs, max_step=T, device=cuda)
        algo = make_algo("dgppo", env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                         action_dim=env.action_dim, n_agents=n, batch_size=64, rnn_step=16, train_steps=100, seed=3,
                         device=cuda)
        infos = []
        for it in range(2):
            r = algo.collect(algo.params, 11 + it, n_env=B)
            infos.append(algo.update(r, it))
        torch.cuda.synchronize()
        return algo, infos

    a0, i0 = run("0")
    a1, i1 = run("1")
    assert a0._mbg is None and a1._mbg is not None  # the graph path really ran
    for name in ("Vl", "Vh", "policy"):
        o0, o1 = a0.opt[name], a1.opt[name]
        assert torch.equal(o0.ps.flat, o1.ps.flat), name
        assert torch.equal(o0.m, o1.m) and torch.equal(o0.v, o1.v) and torch.equal(o0.state, o1.state), name
    for d0, d1 in zip(i0, i1):
        assert d0.keys() == d1.keys()
        for k in d0:
            assert d0[k] == d1[k] or (np.isnan(d0[k]) and np.isnan(d1[k])), k


def test_graph_replay_after_workspace_growth(cuda, monkeypatch):
    """VERDICT r5 next 2 (the round-5 graph-replay fault): capture the minibatch hipGraphs, then grow EVERY
    workspace slot (K.workspace) on the streams the graphs were captured on, and hand the memory a freed buffer would
    return to new sentinel tensors on the same streams; the replayed update must leave the sentinels untouched and
    give parameters, Adam state and info bit-identical to the eager path.  Once the graphs are gone, the kept buffers
    that only they referenced are released."""
    import gc
    import weakref

    from dgppo_fov_amd.nn import kernels as K

    eid, n, obs, B, T = "LidarSpread", 3, 2, 8, 32

    def make(flag):
        monkeypatch.setenv("DGPPO_UPDATE_GRAPH", flag)
        env = make_env(eid, n, num_obs=obs, max_step=T, device=cuda)
        return make_algo("dgppo", env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                         action_dim=env.action_dim, n_agents=n, batch_size=64, rnn_step=16, train_steps=100, seed=4,
                         device=cuda)

    a0 = make("0")
    i0 = [a0.update(a0.collect(a0.params, 31 + it, n_env=B), it) for it in range(2)]
    a1 = make("1")
    i1 = [a1.update(a1.collect(a1.params, 31, n_env=B), 0)]
    torch.cuda.synchronize()
    assert a1._mbg is not None
    sentinels, grown = [], 0
    for (dv, slot, handle), t in list(K._WS.items()):
        if dv != str(cuda):
            continue
        with torch.cuda.stream(torch.cuda.ExternalStream(handle, device=cuda)):
            K.workspace(4 * t.numel() + 4096, cuda, slot)
            sentinels.append(torch.full((t.numel(),), 1234.5, device=cuda))  # reuses a freed block, if any
        grown += 1
    del t
    assert grown >= 3  # the slots of the three nets' streams
    i1.append(a1.update(a1.collect(a1.params, 32, n_env=B), 1))  # every minibatch replays
    torch.cuda.synchronize()
    for s in sentinels:
        assert bool((s == 1234.5).all()), "a replay wrote into a freed workspace buffer"
    for name in ("Vl", "Vh", "policy"):
        o0, o1 = a0.opt[name], a1.opt[name]
        assert torch.equal(o0.ps.flat, o1.ps.flat), name
        assert torch.equal(o0.m, o1.m) and torch.equal(o0.v, o1.v) and torch.equal(o0.state, o1.state), name
    for d0, d1 in zip(i0, i1):
        for k in d0:
            assert d0[k] == d1[k] or (np.isnan(d0[k]) and np.isnan(d1[k])), k
    refs = [weakref.ref(g) for g in a1._mbg[1]]
    del a1, a0
    gc.collect()
    assert all(r() is None for r in refs)
    with torch.cuda.stream(torch.cuda.Stream(cuda)):
        K.workspace(1 << 16, cuda, "growth_probe")
    for _, rs in K._WS_KEPT:
        assert any(r() is not None for r in rs)  # nothing is kept for graphs that are gone


@pytest.mark.gpu
@pytest.mark.parametrize("eid,n,obs,graph", [("LidarSpread", 3, 2, "0"), ("LidarSpread", 3, 2, "1"),
                                             ("LidarBicycleTarget", 3, 2, "0"), ("LidarOmniTarget", 3, 2, "0")])
def test_update_grouped_wgrad_bit_identical(cuda, monkeypatch, eid, n, obs, graph):
    """Each net's weight-gradient GEMMs deferred to the end of its backward and launched as one grouped kernel
    (DGPPO_DEFER_WGRAD=1, K.defer_wgrad, dgppo_gemm_wgrad_grouped) give bit-identical parameters, Adam state and
    info to one launch pair per GEMM (=0), eager and graph-replayed minibatches, over two updates."""
    from dgppo_fov_amd.nn import kernels as K

    B, T = 8, 32

    def run(flag):
        monkeypatch.setenv("DGPPO_DEFER_WGRAD", flag)
        monkeypatch.setenv("DGPPO_UPDATE_GRAPH", graph)
        env = make_env(eid, n, num_obs=obs, max_step=T, device=cuda)
        algo = make_algo("dgppo", env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                         action_dim=env.action_dim, n_agents=n, batch_size=64, rnn_step=16, train_steps=100, seed=5,
                         device=cuda)
        infos = []
        calls = []
        real = K.flush_wgrad

        def counting(device, key=None):
            calls.append(len(K._DEFER.get(K._lib.stream_handle(device) if key is None else key) or ()))
            return real(device, key)

        monkeypatch.setattr(K, "flush_wgrad", counting)
        for it in range(2):
            r = algo.collect(algo.params, 21 + it, n_env=B)
            infos.append(algo.update(r, it))
        torch.cuda.synchronize()
        monkeypatch.setattr(K, "flush_wgrad", real)
        return algo, infos, calls

    a0, i0, c0 = run("0")
    a1, i1, c1 = run("1")
    assert not any(c0) and sum(c1) > 0  # the grouped launches really ran
    for name in ("Vl", "Vh", "policy"):
        o0, o1 = a0.opt[name], a1.opt[name]
        assert torch.equal(o0.ps.flat, o1.ps.flat), name
        assert torch.equal(o0.m, o1.m) and torch.equal(o0.v, o1.v) and torch.equal(o0.state, o1.state), name
    for d0, d1 in zip(i0, i1):
        assert d0.keys() == d1.keys()
        for k in d0:
            assert d0[k] == d1[k] or (np.isnan(d0[k]) and np.isnan(d1[k])), k

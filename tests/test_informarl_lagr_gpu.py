"""InforMARL-Lagr: the global-info cost critic (VhGlobalNet) against the float64 oracle
(values, final carries, every parameter gradient), the three Lagrangian kernels against the NumPy
restatement of informarl_lagr.py:193-305, and one full update: Vh prepass, clipped-cost GAE targets,
advantages, the Vh minibatch gradient (16-step chunks from zero carries) and the multiplier step."""
import numpy as np
import pytest
import torch

from dgppo_fov_amd.algo import make_algo
from dgppo_fov_amd.algo.module.nets import VhGlobalNet
from dgppo_fov_amd.nn import kernels as K
from oracle import nets as ON
from oracle import nets_t as R

from test_nets_gpu import CASES, DENSE, OMNI, _close, _grad_close, _graphs, _walk

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("carry", [0, 1])
@pytest.mark.parametrize("eid,n,obs", CASES[:3] + CASES[4:] + OMNI[:1] + DENSE)
def test_vh_global_seq_fwd_bwd(cuda, eid, n, obs, carry):
    S, L, nh = 3, 4, 2
    env, gb, host = _graphs(cuda, eid, n, obs, S, L, seed=13)
    net = VhGlobalNet(env.node_dim, n, nh, cuda, seed=8, edge_dim=env.edge_dim)
    rng = np.random.default_rng(5)
    h0 = (rng.standard_normal((S * n, 64)) * 0.5).astype(np.float32) if carry else None
    out, hT, cache = net.seq_fwd(gb, S, L, h0=None if h0 is None else torch.from_numpy(h0).to(cuda))
    p = R.to_t(net.flax(), requires_grad=True)
    rout, rh = R.vh_global_seq(p, host, S, L, n, h0=None if h0 is None else h0.reshape(S, n, 64), return_h=True)
    torch.cuda.synchronize()
    _close(out.cpu().numpy(), rout.detach().numpy().reshape(-1, nh), what="Vh (global info)")
    _close(hT.cpu().numpy(), rh.detach().numpy().reshape(S * n, 64), what="final carries")
    w = rng.standard_normal(rout.shape)
    (rout * torch.tensor(w)).sum().backward()
    net.ps.zero_grad()
    net.seq_bwd(cache, torch.tensor(w.reshape(-1, nh), dtype=torch.float32, device=cuda))
    torch.cuda.synchronize()
    net.ps.swap_views()
    g = net.flax()
    net.ps.swap_views()
    for path, a, b in _walk(g, R.grads(p)):
        _grad_close(a, b, "Vh grad " + path)


def test_lagr_kernels(cuda):
    rng = np.random.default_rng(0)
    B, T, n, nh = 5, 40, 3, 2
    c = rng.standard_normal((B, T, n, nh)).astype(np.float32)
    y = torch.empty_like(torch.from_numpy(c)).to(cuda)
    K.clip_min0(torch.from_numpy(c).to(cuda), y)
    Ql = rng.standard_normal((B, T)).astype(np.float32)
    Vl = rng.standard_normal((B, T + 1)).astype(np.float32)
    Qh = rng.standard_normal((B, T, n, nh)).astype(np.float32)
    Vh = rng.standard_normal((B, T + 1, n, nh)).astype(np.float32)
    lagr = rng.uniform(0.1, 1.5, (n, nh)).astype(np.float32)
    d = lambda x: torch.from_numpy(x).to(cuda)  # noqa: E731
    A, Ah = torch.empty((B, T, n), device=cuda), torch.empty((B, T, n, nh), device=cuda)
    K.lagr_advantages(d(Ql), d(Vl), d(Qh), d(Vh), d(lagr), A, Ah)
    torch.cuda.synchronize()
    assert np.array_equal(y.cpu().numpy(), np.maximum(c, 0))
    A_ref, Ah_ref = ON.lagr_advantages(Ql, Vl, Qh, Vh, lagr)
    np.testing.assert_allclose(Ah.cpu().numpy(), Ah_ref, rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(A.cpu().numpy(), A_ref, rtol=1e-5, atol=1e-5)
    # the multiplier step: lr large enough that one multiplier clamps at zero
    lp = rng.standard_normal((B, T, n)).astype(np.float32) * 0.1
    lp_old = lp + rng.standard_normal((B, T, n)).astype(np.float32) * 0.1
    Ahs = Ah_ref.astype(np.float32)
    Vhs = Vh[:, :T].copy()
    Vhs[..., 0, 0] = -400.0  # drives agent 0 / cost 0 negative: relu clamps
    for lr in (1e-7, 1.0):
        lg = d(lagr.copy())
        mean = torch.empty(1, device=cuda)
        K.lagr_update(d(lp), d(lp_old), d(Vhs), d(Ahs), lg, mean, B * T, 0.99, lr)
        torch.cuda.synchronize()
        ref = ON.lagr_update(lagr, lp, lp_old, Vhs, Ahs, 0.99, lr)
        np.testing.assert_allclose(lg.cpu().numpy(), ref, rtol=1e-6, atol=1e-7 if lr < 1 else 1e-5)
        np.testing.assert_allclose(mean.item(), lg.cpu().numpy().mean(), rtol=1e-6)
    assert ref[0, 0] == 0.0


@pytest.mark.parametrize("eid,n,obs", [("LidarSpread", 3, 2), ("LidarBicycleTarget", 3, 2)])
def test_informarl_lagr_update(cuda, eid, n, obs):
    from dgppo_fov_amd.env import make_env

    B, T, L = 4, 32, 16
    env = make_env(eid, n, num_obs=obs, max_step=T, device=cuda)
    algo = make_algo("informarl_lagr", env=env, node_dim=env.node_dim, edge_dim=env.edge_dim,
                     state_dim=env.state_dim, action_dim=env.action_dim, n_agents=n, batch_size=B * T // 2,
                     rnn_step=L, lagr_init=0.5, lr_lagr=1e-2, seed=3, device=cuda)
    assert isinstance(algo.Vh, VhGlobalNet) and algo.config["lagr_init"] == 0.5
    roll = algo.collect(algo.params, 4, n_env=B)
    p_vh = R.to_t(algo.Vh.flax())
    vh_sz, vl_sz = algo.Vh.ps.size, algo.Vl.ps.size
    p_vh_grad = R.to_t(algo.Vh.flax(), requires_grad=True)
    algo.trace = {}
    info = algo.update(roll, 0)
    torch.cuda.synchronize()
    tr = algo.trace
    nh = env.n_cost
    # Vh prepass: whole-episode scan from zero carries + the final value from the last carries
    G = roll.graph
    host = {k: getattr(G, f).cpu().numpy().reshape((B * T,) + tuple(getattr(G, f).shape[2:]))
            for k, f in (("nodes", "nodes"), ("edges", "edges"), ("receivers", "receivers"), ("senders", "senders"))}
    with torch.no_grad():
        rv, rh = R.vh_global_seq(p_vh, host, B, T, n, return_h=True)
        ng = roll.next_graph
        last = {k: getattr(ng, f)[:, -1].cpu().numpy() for k, f in
                (("nodes", "nodes"), ("edges", "edges"), ("receivers", "receivers"), ("senders", "senders"))}
        rf = R.vh_global_seq(p_vh, last, B, 1, n, h0=rh)
    Vh_ref = torch.cat([rv, rf], 1).numpy()
    Vh = tr["Vh"].double().cpu().numpy()
    _close(Vh, Vh_ref, what="Vh prepass")
    # GAE on max(costs, 0) with the GPU's own values, then the advantages
    assert np.array_equal(tr["hs"].cpu().numpy(), np.maximum(roll.costs.cpu().numpy(), 0))
    Vl = tr["Vl"].double().cpu().numpy()
    hs = tr["hs"].double().cpu().numpy()
    l = -roll.rewards.double().cpu().numpy()
    gae = [ON.compute_dec_ocp_gae(hs[b], l[b], Vh[b], Vl[b], algo.gamma, algo.gae_lambda) for b in range(B)]
    np.testing.assert_allclose(tr["Qh"].cpu().numpy(), np.stack([x[0] for x in gae]), rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(tr["Ql"].cpu().numpy(), np.stack([x[1] for x in gae]), rtol=1e-4, atol=1e-4)
    A_ref, Ah_ref = ON.lagr_advantages(tr["Ql"].cpu().numpy(), Vl, tr["Qh"].cpu().numpy(), Vh,
                                       tr["lagr0"].cpu().numpy())
    np.testing.assert_allclose(tr["Ah"].cpu().numpy(), Ah_ref, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(tr["A"].cpu().numpy(), A_ref, rtol=1e-4, atol=1e-4)
    # minibatch 0's Vh gradient: l2 to Qh over 16-step chunks from zero carries (informarl_lagr.py:246-280)
    assert len(tr["mb"]) == 2
    mb0 = tr["mb"][0]
    envs = mb0["envs"]
    Bm = len(envs)
    hm = {k: v.reshape((B, T) + v.shape[1:])[envs].reshape((-1,) + v.shape[1:]) for k, v in host.items()}
    S = Bm * T // L
    out = R.vh_global_seq(p_vh_grad, hm, S, L, n)
    qh = torch.as_tensor(tr["Qh"].cpu().numpy()[envs].reshape(S, L, n, nh), dtype=torch.float64)
    (0.5 * (out - qh) ** 2).mean().backward()
    gflat = mb0["grad"][vl_sz:vl_sz + vh_sz]
    algo.Vh.ps.grad.copy_(gflat)
    algo.Vh.ps.swap_views()
    g = algo.Vh.flax()
    algo.Vh.ps.swap_views()
    for path, a, b in _walk(g, R.grads(p_vh_grad)):
        _grad_close(a, b, "Vh minibatch grad " + path)
    # the multiplier step after each minibatch, fed the GPU's log pi under the updated policy
    lagr = tr["lagr0"].cpu().numpy().astype(np.float64)
    Vh_T = tr["Vh"].cpu().numpy()[:, :T]
    Ah = tr["Ah"].cpu().numpy()
    lp_old = roll.log_pis.cpu().numpy()
    for mb in tr["mb"]:
        e = mb["envs"]
        lp_new = mb["lp_new"].cpu().numpy().reshape(len(e), T, n)
        lagr = ON.lagr_update(lagr, lp_new, lp_old[e], Vh_T[e], Ah[e], algo.gamma, algo.lr_lagr)
        np.testing.assert_allclose(mb["lagr"].cpu().numpy(), lagr, rtol=1e-5, atol=1e-6)
        lagr = mb["lagr"].cpu().numpy().astype(np.float64)
    assert abs(info["policy/lagr_mean"] - float(lagr.mean())) < 1e-6
    for k in ("Vl/loss", "Vh/loss", "Vh/grad_norm", "Vh/has_nan", "policy/loss", "policy/grad_norm"):
        assert np.isfinite(info[k]), k

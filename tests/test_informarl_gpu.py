"""InforMARL: its two extra kernels against the NumPy restatement of
informarl.py:329-337, and one full update whose GAE targets / advantages are checked against the
oracle's compute_dec_ocp_gae fed the GPU's own Vl (the networks, GAE kernel, losses and Adam it shares
with DGPPO are covered by test_nets_gpu.py / test_update_gpu.py)."""
import numpy as np
import pytest
import torch

from dgppo_fov_amd.algo import make_algo
from dgppo_fov_amd.env import make_env
from dgppo_fov_amd.nn import kernels as K
from oracle import env as OE
from oracle import nets as ON

pytestmark = pytest.mark.gpu


def test_shaped_loss_and_advantages_kernels(cuda):
    rng = np.random.default_rng(0)
    B, T, n, nh = 5, 33, 4, 2
    r = rng.standard_normal((B, T)).astype(np.float32)
    c = rng.standard_normal((B, T, n, nh)).astype(np.float32)
    l = torch.empty((B, T), device=cuda)
    K.cost_shaped_loss(torch.from_numpy(r).to(cuda), torch.from_numpy(c).to(cuda), 0.7, l)
    Ql = rng.standard_normal((B, T)).astype(np.float32)
    Vl = rng.standard_normal((B, T + 1)).astype(np.float32)
    A = torch.empty((B, T, n), device=cuda)
    K.informarl_advantages(torch.from_numpy(Ql).to(cuda), torch.from_numpy(Vl).to(cuda), A)
    torch.cuda.synchronize()
    np.testing.assert_allclose(l.cpu().numpy(), ON.informarl_shaped_l(r, c, 0.7), rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(A.cpu().numpy(), ON.informarl_advantages(Ql, Vl, n), rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("eid,n,obs", [("LidarSpread", 3, 2), ("LidarOmniTarget", 3, 2)])
def test_informarl_update(cuda, eid, n, obs):
    B, T, L = 4, 32, 16
    env = make_env(eid, n, num_obs=obs, max_step=T, device=cuda)
    algo = make_algo("informarl", env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                     action_dim=env.action_dim, n_agents=n, batch_size=B * T // 2, rnn_step=L, train_steps=100,
                     cost_weight=0.3, cost_schedule=True, seed=1, device=cuda)
    assert algo.cost_weight_at(10) == 0.3 and algo.cost_weight_at(60) == 1.5 and algo.cost_weight_at(80) == 7.5
    roll = algo.collect(algo.params, 3, n_env=B)
    before = {k: o.ps.flat.clone() for k, o in algo.opt.items()}
    algo.trace = {}
    info = algo.update(roll, 60)
    torch.cuda.synchronize()
    tr = algo.trace
    Vl = tr["Vl"].double().cpu().numpy()
    l_ref = ON.informarl_shaped_l(roll.rewards.cpu().numpy(), roll.costs.cpu().numpy(), 1.5)
    np.testing.assert_allclose(tr["l"].cpu().numpy(), l_ref, rtol=1e-5, atol=1e-5)
    costs = roll.costs.double().cpu().numpy()
    Ql_ref = np.stack([ON.compute_dec_ocp_gae(costs[b], l_ref[b], np.repeat(np.repeat(Vl[b][:, None, None], n, 1),
                                                                          env.n_cost, 2), Vl[b], algo.gamma,
                                              algo.gae_lambda)[1] for b in range(B)])
    np.testing.assert_allclose(tr["Ql"].cpu().numpy(), Ql_ref, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(tr["A"].cpu().numpy(), ON.informarl_advantages(tr["Ql"].cpu().numpy(), Vl, n),
                               rtol=1e-4, atol=1e-4)
    assert len(tr["mb"]) == 2
    for k in ("Vl/loss", "policy/loss", "policy/entropy", "Vl/grad_norm", "policy/grad_norm"):
        assert np.isfinite(info[k]), k
    assert "Vh/loss_Vh" not in info
    assert not torch.equal(before["Vl"], algo.opt["Vl"].ps.flat) and not torch.equal(before["policy"],
                                                                                      algo.opt["policy"].ps.flat)
    assert torch.equal(before["Vh"], algo.opt["Vh"].ps.flat)  # allocated, never stepped


@pytest.mark.parametrize("eid,n,obs", [("LidarSpread", 3, 2), ("MPESpread", 3, 3)])
def test_hcbfcrpo_update(cuda, eid, n, obs):
    """HCBF-CRPO: Vh = the env's cost of each graph (the last next-graph's cost bit-exact vs the oracle
    env), GAE targets and the merged CBF advantage vs the oracle, Vl and policy stepped."""
    B, T, L = 4, 32, 16
    env = make_env(eid, n, num_obs=obs, max_step=T, device=cuda)
    algo = make_algo("hcbfcrpo", env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                     action_dim=env.action_dim, n_agents=n, batch_size=B * T // 2, rnn_step=L, train_steps=100,
                     seed=2, device=cuda)
    roll = algo.collect(algo.params, 5, n_env=B)
    algo.trace = {}
    info = algo.update(roll, 10)
    torch.cuda.synchronize()
    tr = algo.trace
    Vh = tr["Vh"].cpu().numpy()
    assert np.array_equal(Vh[:, :T], roll.costs.cpu().numpy())
    spec = OE.Spec(eid, n, obs)
    ng = roll.next_graph
    st = ng.states[:, -1].cpu().numpy()
    if spec.engine == OE.ENGINE_MPE:
        third = st[:, 2 * n:2 * n + obs]
    else:
        third = ng.env_states.obstacle.packed[:, -1].cpu().numpy()
    ref_cost = OE.env_step(spec, st, third, np.zeros((B, n, env.action_dim), np.float32))["cost"]
    assert np.array_equal(Vh[:, T], ref_cost)
    Vl = tr["Vl"].double().cpu().numpy()
    costs = roll.costs.double().cpu().numpy()
    l = -roll.rewards.double().cpu().numpy()
    Ql_ref = np.stack([ON.compute_dec_ocp_gae(costs[b], l[b], Vh[b].astype(np.float64), Vl[b], algo.gamma,
                                              algo.gae_lambda)[1] for b in range(B)])
    np.testing.assert_allclose(tr["Ql"].cpu().numpy(), Ql_ref, rtol=1e-4, atol=1e-4)
    A_ref, safe_ref, deriv = ON.merged_cbf_advantages(tr["Ql"].cpu().numpy(), Vl, Vh, n, env.dt, algo.alpha,
                                                      algo.cbf_eps, algo.cbf_weight_at(10))
    robust = np.abs(deriv).min(-1) > 1e-3  # where the safe-set decision is not an fp32 coin flip
    np.testing.assert_allclose(tr["A"].cpu().numpy()[robust], A_ref[robust], rtol=1e-3, atol=1e-3)
    assert abs(info["eval/safe_data"] - safe_ref) <= (~robust).mean() + 1e-6
    for k in ("Vl/loss", "policy/loss", "Vl/grad_norm", "policy/grad_norm"):
        assert np.isfinite(info[k]), k

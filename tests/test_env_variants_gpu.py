"""GPU parity for the reference's env variants: LidarLine, MPELine, MPEFormation,
MPECorridor, MPEConnectSpread on the variant kernels (csrc/env_step.hip namespace var) against
oracle/env_variants.py.  Bar: BIT-EXACT reset graphs, obstacle records, step chains (graph, reward, cost),
as for the base envs (tests/test_env_gpu.py); plus one DGPPO collect + update on two variants."""
import numpy as np
import pytest
import torch

from dgppo_fov_amd.algo import make_algo
from dgppo_fov_amd.env import make_env
from oracle import env as O

from test_env_gpu import _np, assert_graph_equal, oracle_third

pytestmark = pytest.mark.gpu

CONFIGS = [
    ("LidarLine", 5, 3, 24),
    ("LidarLine", 3, 0, 8),
    ("MPELine", 3, 3, 24),  # n <= 3: interior goals, uniform first landmark
    ("MPELine", 5, 3, 24),
    ("MPEFormation", 4, 3, 24),
    ("MPEFormation", 6, 0, 8),
    ("MPECorridor", 3, 2, 24),
    ("MPECorridor", 5, 7, 8),  # n_obs forced to 2
    ("MPEConnectSpread", 3, 1, 16),
]
IDS = [f"{c[0]}-n{c[1]}-o{c[2]}" for c in CONFIGS]


@pytest.mark.parametrize("cfg", CONFIGS, ids=IDS)
def test_variant_reset_matches_oracle(cuda, cfg):
    eid, n, obs, B = cfg
    env = make_env(eid, n, num_obs=obs, device=cuda)
    spec = O.Spec(eid, n, obs)
    assert (env.n_nodes, env.n_edges, env.n_cost, env.num_goals) == (spec.n_nodes, spec.n_edges, spec.n_cost, spec.ng)
    g = env.reset(key=4321, n_env=B)
    torch.cuda.synchronize()
    ag, gl, third = O.env_reset(spec, 4321, B)
    ref = O.initial_graph(spec, ag, gl, third)
    assert_graph_equal(g, ref, "reset")
    if spec.engine != O.ENGINE_MPE and spec.n_obs > 0:
        np.testing.assert_array_equal(_np(g.env_states.obstacle.packed), third)
    np.testing.assert_array_equal(_np(g.node_type[0]), O.node_type(spec))


@pytest.mark.parametrize("cfg", CONFIGS, ids=IDS)
def test_variant_step_chain_matches_oracle(cuda, cfg):
    eid, n, obs, B = cfg
    env = make_env(eid, n, num_obs=obs, device=cuda)
    spec = O.Spec(eid, n, obs)
    g = env.reset(key=77, n_env=B)
    rng = np.random.default_rng(3)
    states = _np(g.states)
    third = oracle_third(spec, g)
    for t in range(5):
        a = rng.uniform(-1.5, 1.5, (B, n, 2)).astype(np.float32)
        res = env.step(g, torch.from_numpy(a).to(cuda))
        ref = O.env_step(spec, states, third, a)
        torch.cuda.synchronize()
        assert_graph_equal(res.graph, ref, f"step{t}")
        np.testing.assert_array_equal(_np(res.cost), ref["cost"], err_msg=f"cost step{t}")
        np.testing.assert_array_equal(_np(res.reward), ref["reward"], err_msg=f"reward step{t}")
        g, states = res.graph, ref["states"]


def test_connect_cost_and_corridor_edges_hand_cases(cuda):
    """Known answers: three agents in a row 0.3 apart -> connectivity cost 0.3 - 0.45 = -0.15 -> -0.65
    after the margin; pull the last one to 0.6 away -> +0.15 -> +0.65 for EVERY agent.  Corridor obstacle
    edges are kept at any distance (comm_radius * 100)."""
    env = make_env("MPEConnectSpread", 3, device=cuda)
    g = env.reset(key=1, n_env=2)
    st = _np(g.states).copy()
    st[:, :3, :2] = np.array([[0.2, 0.1], [0.5, 0.1], [0.8, 0.1]], np.float32)
    st[1, 2, 0] = 1.1
    gin = env._assemble(g.nodes, g.edges, torch.from_numpy(st).to(cuda), g.receivers, g.senders, None)
    res = env.step(gin, torch.zeros((2, 3, 2), device=cuda))
    c = _np(res.cost)
    np.testing.assert_allclose(c[0, :, 2], -0.65, atol=1e-6)
    np.testing.assert_allclose(c[1, :, 2], np.float32(0.6) - np.float32(0.45) + np.float32(0.5), atol=1e-6)
    env = make_env("MPECorridor", 3, device=cuda)
    g = env.reset(key=2, n_env=1)
    E0 = 3 * 3 + 3 * 3  # agent-agent + agent-goal blocks
    recv = _np(g.receivers)[0, E0:]
    assert (recv != env.n_nodes - 1).all()  # every agent-obstacle edge present


@pytest.mark.parametrize("eid,n,obs", [("MPEConnectSpread", 3, 1), ("LidarLine", 4, 3)])
def test_dgppo_trains_on_variant(cuda, eid, n, obs):
    B, T = 8, 32
    env = make_env(eid, n, num_obs=obs, max_step=T, device=cuda)
    algo = make_algo("dgppo", env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                     action_dim=env.action_dim, n_agents=n, batch_size=B * T // 2, rnn_step=16, seed=0, device=cuda)
    roll = algo.collect(algo.params, 1, n_env=B)
    assert roll.costs.shape == (B, T, n, env.n_cost)
    before = algo.actor.ps.flat.clone()
    info = algo.update(roll, 0)
    torch.cuda.synchronize()
    for k in ("Vl/loss", "policy/loss", "Vh/loss_Vh"):
        assert np.isfinite(info[k]), k
    assert not torch.equal(before, algo.actor.ps.flat)

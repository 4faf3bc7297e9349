"""GPU parity for the VMAS contact-physics envs: VMASWheel and VMASReverseTransport
on csrc/vmas.hip (through the dgppo_env_* C-ABI) against oracle/vmas.py.  Bar: BIT-EXACT graphs (nodes,
edges, states, receivers, senders), env records, rewards and costs, for resets, step chains from sampled
and from hand-placed contact states (every contact branch: sphere-line with torque and the angular-velocity
clamp, box sides with the closest-side search), and the persistent rollout kernel against per-step launches.
Then DGPPO / InforMARL collect + update on both (the networks on the 13 / 20-wide VMAS nodes are checked
against the float64 oracle in tests/test_nets_gpu.py, VMAS cases)."""
import math

import numpy as np
import pytest
import torch

from dgppo_fov_amd.env import make_env
from oracle import vmas as V

from test_env_gpu import _np, assert_graph_equal

pytestmark = pytest.mark.gpu

KINDS = [V.WHEEL, V.TRANSPORT]


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("seed,B,offset", [(1234, 96, 0), (2 ** 40 + 7, 33, 5)])
def test_vmas_reset_matches_oracle(cuda, kind, seed, B, offset):
    env = make_env(kind, 3, device=cuda)
    assert (env.n_nodes, env.n_edges, env.node_dim, env.n_cost) == (4, 9, V.NODE_DIM[kind], 2)
    g = env.reset(key=seed, n_env=B, env_offset=offset)
    torch.cuda.synchronize()
    st, rec = V.reset(kind, seed, B, offset)
    np.testing.assert_array_equal(_np(g.env_states.record), rec)
    assert_graph_equal(g, V.initial_graph(kind, st, rec), f"{kind} reset")
    np.testing.assert_array_equal(_np(g.node_type[0]), [0, 0, 0, -1])


def _step_chain(cuda, env, kind, g, steps, rng, lim=1.5):
    st, rec = _np(g.states), _np(g.env_states.record)
    B = st.shape[0]
    contact_seen = 0
    for t in range(steps):
        a = rng.uniform(-lim, lim, (B, 3, 2)).astype(np.float32)
        res = env.step(g, torch.from_numpy(a).to(cuda))
        ref = V.step(kind, st, rec, a)
        torch.cuda.synchronize()
        assert_graph_equal(res.graph, ref, f"{kind} step {t}")
        np.testing.assert_array_equal(_np(res.reward), ref["reward"], err_msg=f"reward step {t}")
        np.testing.assert_array_equal(_np(res.cost), ref["cost"], err_msg=f"cost step {t}")
        if kind == V.WHEEL:
            contact_seen += int((np.abs(ref["nodes"][:, :3, 7:9]) > 0).any(-1).sum())
        g, st = res.graph, ref["states"]
    return g, contact_seen


@pytest.mark.parametrize("kind", KINDS)
def test_vmas_step_chain_matches_oracle(cuda, kind):
    env = make_env(kind, 3, device=cuda)
    g = env.reset(key=77, n_env=12)
    _step_chain(cuda, env, kind, g, 8, np.random.default_rng(3))


def _placed_states(kind, B, rng):
    """Pre-step states with agents inside the contact band of the line / box walls."""
    st, rec = V.reset(kind, 99, B)
    for b in range(B):
        if kind == V.WHEEL:
            rot = np.float32(rng.uniform(-np.pi, np.pi))
            st[b, 3, 0] = rot
            st[b, 3, 1] = np.float32(rng.choice([0.0, 0.59, -0.59, 0.3]))
            for i in range(3):  # a point along the line, offset sideways by 0.01 .. 0.04 (contact below ~0.0367)
                u = rng.uniform(-1.1, 1.1)
                off = rng.uniform(0.0, 0.04) * rng.choice([-1, 1])
                st[b, i, 0] = np.float32(np.cos(rot) * u - np.sin(rot) * off)
                st[b, i, 1] = np.float32(np.sin(rot) * u + np.cos(rot) * off)
                st[b, i, 2:] = rng.uniform(-0.3, 0.3, 2).astype(np.float32)
        else:
            bx, by = st[b, 3, 0], st[b, 3, 1]
            st[b, 3, 2:] = rng.uniform(-0.2, 0.2, 2).astype(np.float32)
            for i in range(3):  # near a wall (inside or outside) or a corner
                side = rng.integers(4)
                along = rng.uniform(-0.35, 0.35)
                off = 0.3 + rng.uniform(-0.04, 0.04)
                dx, dy = [(off, along), (-off, along), (along, off), (along, -off)][side]
                st[b, i, 0], st[b, i, 1] = np.float32(bx + dx), np.float32(by + dy)
                st[b, i, 2:] = rng.uniform(-0.3, 0.3, 2).astype(np.float32)
    return st, rec


@pytest.mark.parametrize("kind", KINDS)
def test_vmas_contact_states_match_oracle(cuda, kind):
    """Hand-placed contact configurations (GPU and oracle start from the same uploaded state)."""
    B = 24
    rng = np.random.default_rng(11)
    st, rec = _placed_states(kind, B, rng)
    env = make_env(kind, 3, device=cuda)
    g0 = env.reset(key=99, n_env=B)
    g0.states.copy_(torch.from_numpy(st))
    g0.env_states.record.copy_(torch.from_numpy(rec))
    g, contacts = _step_chain(cuda, env, kind, g0, 4, rng, lim=1.0)
    if kind == V.WHEEL:
        assert contacts >= B // 4  # the contact branch ran (last-world-step forces in the node columns 7:9)
    else:
        ref = V.step(kind, st, rec, np.zeros((B, 3, 2), np.float32))
        moved = np.abs(ref["states"][:, 3, 2:] - st[:, 3, 2:] * np.float32(0.75 ** 4)).max()
        assert moved > 1e-4  # the agents pushed the box


@pytest.mark.parametrize("kind", KINDS)
def test_vmas_rollout_kernel_matches_steps(cuda, kind):
    """The persistent rollout kernel (state in registers for all T steps) == T step launches, bit for bit,
    through the RolloutEngine's time-major buffers (reset_states + rollout_into)."""
    env = make_env(kind, 3, device=cuda)
    B, T = 200, 40
    rng = np.random.default_rng(5)
    acts = torch.from_numpy(rng.uniform(-1.2, 1.2, (T, B, 3, 2)).astype(np.float32)).to(cuda)
    buf = env.empty_graph((T + 1, B), cuda)
    rec = torch.empty((B, 1, 8), device=cuda)
    rew = torch.empty((T, B), device=cuda)
    cost = torch.empty((T, B, 3, 2), device=cuda)
    g0 = env._assemble(buf.nodes[0], buf.edges[0], buf.states[0], buf.receivers[0], buf.senders[0], None)
    env.reset_states(31, n_env=B, out=g0, obstacles_out=rec)
    env.rollout_into(buf, rec, acts, rew, cost, rebuild_first=True)
    g = env.reset(key=31, n_env=B)
    for t in range(T):
        res = env.step(g, acts[t])
        torch.cuda.synchronize()
        for f in ("nodes", "edges", "states", "receivers", "senders"):
            assert torch.equal(getattr(res.graph, f), getattr(buf, f)[t + 1]), (t, f)
        assert torch.equal(res.reward, rew[t]) and torch.equal(res.cost, cost[t]), t
        g = res.graph
    # and the first steps against the oracle (it reads the graph the kernels start from)
    st, r = V.reset(kind, 31, 8)
    graphs, rr, cc = V.rollout(kind, st, r, _np(acts[:3, :8]))
    for t in range(3):
        np.testing.assert_array_equal(_np(buf.nodes[t + 1, :8]), graphs[t]["nodes"])
    np.testing.assert_array_equal(_np(rew[:3, :8]), rr)
    np.testing.assert_array_equal(_np(cost[:3, :8]), cc)


def test_vmas_env_states_views(cuda):
    w = make_env("VMASWheel", 3, device=cuda)
    g = w.reset(key=3, n_env=4)
    es = g.env_states
    assert es.a_pos.shape == (4, 3, 2) and es.line_angle.shape == (4,) and es.a_contact_force.shape == (4, 3, 2)
    assert torch.equal(es.goal_angle, g.env_states.record[:, 0, 0])
    t = make_env("VMASReverseTransport", 3, device=cuda)
    g = t.reset(key=3, n_env=4)
    assert g.env_states.o_pos.shape == (4, 3, 2) and g.env_states.box_pos.shape == (4, 2)
    # every agent starts inside the box (vmas_reverse_transport.py:114-123)
    rel = (g.env_states.a_pos - g.env_states.box_pos[:, None]).abs()
    assert (rel <= 0.3).all()
    with pytest.raises(AssertionError):
        make_env("VMASWheel", 4, device=cuda)


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("algo", ["dgppo", "informarl"])
def test_vmas_collect_update(cuda, kind, algo):
    """One collect + update of DGPPO / InforMARL on a VMAS env: finite losses, parameters move."""
    from dgppo_fov_amd.algo import make_algo

    env = make_env(kind, 3, max_step=32, device=cuda)
    B, T = 16, 32
    al = make_algo(algo, env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                   action_dim=env.action_dim, n_agents=3, batch_size=B * T // 2, rnn_step=16, seed=0, device=cuda)
    r = al.collect(al.params, 0, n_env=B)
    assert r.costs.shape == (B, T, 3, 2)
    assert torch.isfinite(r.rewards).all() and torch.isfinite(r.costs).all()
    before = al.actor.ps.flat.clone()
    info = al.update(r, 0)
    torch.cuda.synchronize()
    assert all(math.isfinite(v) for v in info.values() if isinstance(v, float)), info
    assert not torch.equal(before, al.actor.ps.flat)


@pytest.mark.parametrize("kind", KINDS)
def test_vmas_train_then_test_entry_points(cuda, tmp_path, monkeypatch, capsys, kind):
    """train.py / test.py on a VMAS env (the reference's `--env VMASWheel -n 3` CLI)."""
    import glob
    import sys

    from test_train_gpu import _entry

    test_py, train_py = _entry("test"), _entry("train")
    argv = ["train.py", "--env", kind, "-n", "3", "--obs", "0", "--algo", "dgppo", "--steps", "2", "--n-env-train", "8",
            "--batch-size", "256", "--n-env-test", "4", "--eval-interval", "1", "--save-interval", "2",
            "--log-dir", str(tmp_path)]
    monkeypatch.setattr(sys, "argv", argv)
    train_py.main()
    runs = glob.glob(str(tmp_path / kind / "dgppo" / "seed0_*"))
    assert len(runs) == 1
    capsys.readouterr()
    monkeypatch.setattr(sys, "argv", ["test.py", "--path", runs[0], "--epi", "3", "--max-step", "16", "--no-video"])
    test_py.main()
    out = capsys.readouterr().out
    assert "safe_rate:" in out and out.count("epi: ") == 3

"""Hand-derived known-answer tests that pin the NumPy oracle (oracle/env.py, oracle/math32.py).

The reference ships no tests or golden vectors and JAX is absent, so these
closed-form cases are what pins the restatement (parity unpinned against the reference itself)."""
import numpy as np
import pytest

from oracle import env as O
from oracle import math32 as M

F = np.float32


# ---- math32 ------------------------------------------------------------------------------------
def test_philox_random123_kat():
    # Random123 kat_vectors for philox4x32-10
    assert [int(x) for x in M.philox4x32(0, 0, 0, 0, 0, 0)] == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    f = 0xFFFFFFFF
    assert [int(x) for x in M.philox4x32(f, f, f, f, f, f)] == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]
    got = M.philox4x32(0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344, 0xA4093822, 0x299F31D0)
    assert [int(x) for x in got] == [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def test_uniform_map_matches_jax_definition():
    # jax.random.uniform: bitcast((bits >> 9) | 0x3f800000) - 1, then max(lo, u*(hi-lo)+lo)
    assert M.bits_to_unit(np.uint32(0)) == 0.0
    assert M.bits_to_unit(np.uint32(0xFFFFFFFF)) == F(1.0) - F(2.0 ** -23)
    u = M.uniform(np.uint32(0x80000000), 0.0, 1.5)
    assert u == F(0.5) * F(1.5)


def test_sincos_atan2_accuracy():
    x = np.linspace(-7, 7, 100001).astype(F)
    s, c = M.sincos(x)
    assert np.max(np.abs(s - np.sin(x.astype(np.float64)))) < 1.2e-7
    assert np.max(np.abs(c - np.cos(x.astype(np.float64)))) < 1.2e-7
    y = np.random.default_rng(0).uniform(-1, 1, (2, 50000)).astype(F)
    a = M.atan2(y[0], y[1])
    assert np.max(np.abs(a - np.arctan2(y[0].astype(np.float64), y[1].astype(np.float64)))) < 4e-7
    assert M.atan2(F(0), F(1)) == 0 and abs(M.atan2(F(1), F(0)) - np.pi / 2) < 2e-7


# ---- geometry ------------------------------------------------------------------------------------
def test_ray_thetas_linspace():
    th = O.ray_thetas(32)
    assert th.dtype == F and th.shape == (32,)
    np.testing.assert_allclose(th, np.linspace(-np.pi, np.pi - 2 * np.pi / 32, 32), atol=3e-7)
    assert th[0] == F(-np.pi) and th[-1] == F(np.pi - 2 * np.pi / 32)


def test_rectangle_corners_axis_aligned():
    rec = O.make_rectangles(np.array([[0.8, 0.5]], F), np.array([0.2], F), np.array([0.4], F), np.array([0.0], F))
    pts = rec[0, 8:].reshape(4, 2)
    np.testing.assert_allclose(pts, [[0.9, 0.7], [0.7, 0.7], [0.7, 0.3], [0.9, 0.3]], atol=1e-7)
    assert rec[0, 5] == 1.0 and rec[0, 6] == 0.0


def test_inside_with_radius():
    rec = O.make_rectangles(np.array([0.5, 0.5], F), F(0.2), F(0.2), F(0.0))
    assert O.inside_rect(F(0.5), F(0.5), rec, 0.0)
    assert not O.inside_rect(F(0.65), F(0.5), rec, 0.0)
    assert O.inside_rect(F(0.65), F(0.5), rec, 0.06)  # within r of the right edge
    # corner region: (0.63, 0.63) is 0.03*sqrt(2)=0.0424 from the corner
    assert not O.inside_rect(F(0.63), F(0.63), rec, 0.04)
    assert O.inside_rect(F(0.63), F(0.63), rec, 0.05)


def _lidar_one(pos, rec, k=8):
    hits, alpha = O.lidar(np.asarray(pos, F)[None, None], np.asarray(rec, F)[None], O.ray_table(32, 0.5), k)
    return hits[0, 0], alpha[0, 0]


def test_ray_hits_square_at_known_alpha():
    rec = O.make_rectangles(np.array([[0.8, 0.5]], F), np.array([0.2], F), np.array([0.2], F), np.array([0.0], F))
    hits, alpha = _lidar_one([0.5, 0.5], rec)
    # ray 16 has theta = 0 (up to fp32 rounding of linspace): enters the square at x = 0.7
    assert abs(alpha[16] - 0.4) < 1e-6
    np.testing.assert_allclose(hits[0], [0.7, 0.5], atol=1e-6)
    # only rays pointing at the square hit; all others report alpha = 1e6
    assert np.sum(alpha < 1) >= 3 and np.sum(alpha == F(1e6)) == 32 - np.sum(alpha < 1)


def test_no_hit_gives_far_points_in_ray_order():
    rec = O.make_rectangles(np.array([[1.4, 1.4]], F), np.array([0.1], F), np.array([0.1], F), np.array([0.0], F))
    hits, alpha = _lidar_one([0.2, 0.2], rec)
    assert np.all(alpha == F(1e6))
    tab = O.ray_table(32, 0.5)
    # stable argsort of equal keys = rays 0..7, hit = start + (end - start) * 1e6
    for h in range(8):
        ex = F(0.2) + tab[h, 0]
        np.testing.assert_array_equal(hits[h, 0], F(0.2) + (ex - F(0.2)) * F(1e6))


def test_agent_inside_obstacle_gives_start_points():
    rec = O.make_rectangles(np.array([[0.5, 0.5]], F), np.array([0.3], F), np.array([0.3], F), np.array([0.3], F))
    hits, alpha = _lidar_one([0.5, 0.5], rec)
    assert np.all(alpha == 0)
    np.testing.assert_array_equal(hits, np.full((8, 2), 0.5, F))


# ---- cost / reward / dynamics ---------------------------------------------------------------------
def test_agent_cost_margin():
    spec = O.Spec("LidarSpread", 2, 0)
    agent = np.zeros((2, 2, 4), F)
    agent[0, 1, 0] = 0.08  # d = 0.08 -> 0.1 - 0.08 = 0.02 > 0 -> +0.5
    agent[1, 1, 0] = 0.3  # d = 0.3 -> -0.2 -> -0.7
    c = O.get_cost_lidar(spec, agent, None)
    np.testing.assert_allclose(c[0, :, 0], [0.52, 0.52], atol=1e-6)
    np.testing.assert_allclose(c[1, :, 0], [-0.7, -0.7], atol=1e-6)
    assert np.all(c[..., 1] == F(-0.5))  # no obstacles: 0 - 0.5


def test_mpe_cost_has_no_upper_clip():
    spec = O.Spec("MPESpread", 2, 1)
    agent = np.zeros((1, 2, 4), F)
    agent[0, 1, 0] = 1.0
    obs = np.zeros((1, 1, 4), F)  # obstacle on agent 0 -> 0.1 - 0 + 0.5 = 0.6
    c = O.get_cost_mpe(spec, agent, obs)
    assert abs(c[0, 0, 1] - 0.6) < 1e-6


def test_double_integrator_and_clip():
    spec = O.Spec("LidarSpread", 1, 0)
    x = np.array([[[0.5, 0.5, 0.2, -0.1]]], F)
    a = np.array([[[1.0, -0.5]]], F)
    y = O.step_double_integrator(spec, x, a)
    np.testing.assert_allclose(y[0, 0], [0.5 + 0.2 * 0.03, 0.5 - 0.1 * 0.03, 0.5, -0.25], atol=1e-7)


def test_bicycle_heading_update():
    spec = O.Spec("LidarBicycleTarget", 1, 0)
    x = np.array([[[0.5, 0.5, 1.0, 0.0, 0.4]]], F)  # heading 0, v = 0.4
    a = np.array([[[1.0, 0.0]]], F)
    y = O.step_bicycle(spec, x, a)
    th = 0.4 * 1.0 * 0.03 * 10
    np.testing.assert_allclose(y[0, 0], [0.5 + 0.4 * 0.03, 0.5, np.cos(th), np.sin(th), 0.4], atol=2e-7)


def test_spread_reward_at_goals():
    spec = O.Spec("LidarSpread", 2, 0)
    agent = np.zeros((1, 2, 4), F)
    agent[0, :, :2] = [[0.2, 0.2], [0.9, 0.9]]
    goal = agent.copy()[:, ::-1]  # goals permuted: spread matches each goal to its nearest agent
    a = np.array([[[0.6, 0.8], [0.0, 0.0]]], F)  # |a|^2 = 1 and 0
    r = O.get_reward(spec, agent, goal, a)
    assert abs(r[0] - (-0.0001 * 0.5)) < 1e-9


# ---- graph layout ---------------------------------------------------------------------------------
@pytest.mark.parametrize("eid,n,obs,N,E", [
    ("MPETarget", 3, 0, 7, 12), ("MPESpread", 3, 3, 10, 27), ("LidarSpread", 8, 3, 81, 192),
    ("LidarBicycleTarget", 8, 3, 81, 136), ("LidarSpread", 32, 8, 321, 2304)])
def test_graph_sizes_match_survey(eid, n, obs, N, E):
    s = O.Spec(eid, n, obs)
    assert (s.n_nodes, s.n_edges) == (N, E)


def test_graph_layout_lidar_spread():
    spec = O.Spec("LidarSpread", 2, 1, top_k=2)
    agent = np.zeros((1, 2, 4), F)
    agent[0, 0, :2] = [0.1, 0.1]
    agent[0, 1, :2] = [0.3, 0.1]  # d = 0.2 < 0.5: connected
    goal = np.zeros((1, 2, 4), F)
    goal[0, :, :2] = [[1.0, 1.0], [1.2, 1.0]]
    hits = np.array([[[[0.15, 0.1], [5.0, 5.0]], [[0.3, 0.2], [0.3, 0.9]]]], F)  # (1, n, k, 2)
    g = O.build_graph(spec, agent, goal, hits)
    N, pad = spec.n_nodes, spec.n_nodes - 1
    assert N == 2 + 2 + 4 + 1
    np.testing.assert_array_equal(g["nodes"][0, 0], np.array([0.1, 0.1, 0, 0, 0, 0, 1], F))
    np.testing.assert_array_equal(g["nodes"][0, 2], np.array([1.0, 1.0, 0, 0, 0, 1, 0], F))
    np.testing.assert_array_equal(g["nodes"][0, 4], np.array([0.15, 0.1, 0, 0, 1, 0, 0], F))
    np.testing.assert_array_equal(g["nodes"][0, pad], np.zeros(7))
    np.testing.assert_array_equal(g["states"][0, pad], -np.ones(4))
    # agent-agent: self edges masked to the pad node, 0<->1 connected
    np.testing.assert_array_equal(g["receivers"][0, :4], [pad, 0, 1, pad])
    np.testing.assert_array_equal(g["senders"][0, :4], [pad, 1, 0, pad])
    # agent-goal (spread): all four present
    np.testing.assert_array_equal(g["receivers"][0, 4:8], [0, 0, 1, 1])
    np.testing.assert_array_equal(g["senders"][0, 4:8], [2, 3, 2, 3])
    # agent-lidar: agent 0 hit 0 at d=0.05 (active), hit 1 far (masked); agent 1: d=0.1 and 0.8
    np.testing.assert_array_equal(g["receivers"][0, 8:], [0, pad, 1, pad])
    np.testing.assert_array_equal(g["senders"][0, 8:], [4, pad, 6, pad])
    np.testing.assert_allclose(g["edges"][0, 8], [-0.05, 0, 0, 0], atol=1e-7)


def test_reset_invariants():
    spec = O.Spec("LidarSpread", 4, 3)
    ag, gl, ob = O.env_reset(spec, 7, 6)
    md = F(2.2 * 0.05)
    for b in range(6):
        p = ag[b, :, :2]
        d = np.linalg.norm(p[:, None] - p[None], axis=-1) + np.eye(4) * 10
        assert d.min() > md
        for i in range(4):
            assert not O.inside_rect(p[i, 0], p[i, 1], ob[b], F(2.2 * 0.05 / 2)).any()
        assert np.all((p >= 0) & (p <= 1.5))
        assert np.all(ag[b, :, 2:] == 0)
        assert np.all((ob[b, :, 2:4] >= 0.1) & (ob[b, :, 2:4] <= 0.3))


# ---- Dec-OCP GAE (dgppo/algo/utils.py:11-79, lax.scan(reverse=True) over ts = arange(T)[::-1]) ------
def _gae_inputs(T=12, n=3, nh=2, seed=0):
    rng = np.random.default_rng(seed)
    return (rng.standard_normal((T, n, nh)), rng.standard_normal(T), rng.standard_normal((T + 1, n, nh)),
            rng.standard_normal(T + 1))


def test_gae_ql_is_textbook_td_lambda():
    from oracle.nets import compute_dec_ocp_gae

    hs, l, Vh, Vl = _gae_inputs()
    g, lam = 0.99, 0.95
    T = len(l)
    G = np.zeros(T)
    for t in range(T - 1, -1, -1):
        G[t] = l[t] + g * (Vl[T] if t == T - 1 else (1 - lam) * Vl[t + 1] + lam * G[t + 1])
    _, Ql = compute_dec_ocp_gae(hs, l, Vh, Vl, g, lam)
    np.testing.assert_allclose(Ql, G, rtol=0, atol=1e-12)


def test_gae_lambda_zero_and_one():
    """lambda = 0: every target is the one-step backup; lambda = 1: the full-horizon backup."""
    from oracle.nets import compute_dec_ocp_gae

    hs, l, Vh, Vl = _gae_inputs(T=7, n=2, nh=2, seed=3)
    g = 0.9
    T = len(l)
    Qh, Ql = compute_dec_ocp_gae(hs, l, Vh, Vl, g, 0.0)
    hmax = hs.max(-1, keepdims=True)
    np.testing.assert_allclose(Ql, l + g * Vl[1:], atol=1e-12)
    np.testing.assert_allclose(Qh, np.maximum(hs, (1 - g) * hmax + g * Vh[1:]), atol=1e-12)
    Qh1, Ql1 = compute_dec_ocp_gae(hs, l, Vh, Vl, g, 1.0)
    full_h = Vh[T]
    full_l = Vl[T]
    for t in range(T - 1, -1, -1):
        full_h = np.maximum(hs[t], (1 - g) * hmax[t] + g * full_h)
        full_l = l[t] + g * full_l
        np.testing.assert_allclose(Qh1[t], full_h, atol=1e-12)
        np.testing.assert_allclose(Ql1[t], full_l, atol=1e-12)


def test_gae_two_steps_by_hand():
    from oracle.nets import compute_dec_ocp_gae

    hs, l, Vh, Vl = _gae_inputs(T=2, n=1, nh=2, seed=5)
    g, lam = 0.99, 0.95
    Qh, _ = compute_dec_ocp_gae(hs, l, Vh, Vl, g, lam)
    hm = hs.max(-1, keepdims=True)
    one1 = np.maximum(hs[1], (1 - g) * hm[1] + g * Vh[2])  # time 1: one-step
    one0 = np.maximum(hs[0], (1 - g) * hm[0] + g * Vh[1])
    two0 = np.maximum(hs[0], (1 - g) * hm[0] + g * one1)
    np.testing.assert_allclose(Qh[1], one1, atol=1e-12)
    np.testing.assert_allclose(Qh[0], lam * two0 + (1 - lam) * one0, atol=1e-12)


# ---- LidarOmniTarget (lidar_omni_target.py) ------------------------------------------------------
def _omni_states(spec, agent_rows, hits=None):
    """(1, N, 7) pre-step states: agents, goals at the agents' positions, hits far away."""
    n, N = spec.n, spec.n_nodes
    st = np.zeros((1, N, 7), F)
    st[0, :n] = np.asarray(agent_rows, F)
    st[0, n:2 * n, :2] = st[0, :n, :2]
    st[0, 2 * n:N - 1, :2] = 5.0 if hits is None else hits
    st[0, N - 1] = -1
    return st


def test_omni_fov_costs_by_hand():
    spec = O.Spec("LidarOmniTarget", 2, 1)
    # agent 0 at (0.5, 0.5) facing +x, agent 1 straight ahead at distance 0.3 (in FoV, in range)
    st = _omni_states(spec, [[0.5, 0.5, 1, 0, 0, 0, 0], [0.8, 0.5, 1, 0, 0, 0, 0]])
    c = O.get_cost_omni(spec, st[:, :2], st[:, 4:4 + 16, :2])
    cb = O.omni_cos_fov(spec)
    np.testing.assert_allclose(c[0, 0, 2], cb * F(0.3 + 1e-8) - F(0.3) - F(0.1), atol=1e-6)  # h_angle
    np.testing.assert_allclose(c[0, 0, 3], 0.3 - 0.5 - 0.1, atol=1e-6)  # h_range
    np.testing.assert_allclose(c[0, 0, 4], 0.2 - 0.3 - 0.1, atol=1e-6)  # h_coll_fov
    np.testing.assert_array_equal(c[0, 1, 2:], [-1.0, -1.0, -1.0])  # last agent: safe value -1 - 0.1, clipped
    # agent 1 behind agent 0: angle violated (h_angle = cos_b * 0.3 + 0.3 > 0)
    st = _omni_states(spec, [[0.5, 0.5, 1, 0, 0, 0, 0], [0.2, 0.5, 1, 0, 0, 0, 0]])
    c = O.get_cost_omni(spec, st[:, :2], st[:, 4:4 + 16, :2])
    np.testing.assert_allclose(c[0, 0, 2], min(1.0, cb * 0.3 + 0.3 + 0.1), atol=1e-6)


def test_omni_obstacle_cost_includes_origin_row():
    """type_states(2, N - 2n) asks for one row more than there are hits (the pad node is counted):
    that zero row is the origin, so ||p_i|| enters min_dist_obs."""
    spec = O.Spec("LidarOmniTarget", 2, 1)
    st = _omni_states(spec, [[0.06, 0.08, 1, 0, 0, 0, 0], [1.0, 1.0, 1, 0, 0, 0, 0]])
    c = O.get_cost_omni(spec, st[:, :2], st[:, 4:4 + 16, :2])
    np.testing.assert_allclose(c[0, 0, 1], 0.05 - 0.1 - 0.1, atol=1e-6)  # r - ||p_0 - 0||, margin
    # every agent's hits count, not only its own: put agent 1's first hit next to agent 0
    hits = np.full((16, 2), 5.0, F)
    hits[8] = [0.06 + 0.01, 0.08]
    st = _omni_states(spec, [[0.06, 0.08, 1, 0, 0, 0, 0], [1.0, 1.0, 1, 0, 0, 0, 0]], hits)
    c = O.get_cost_omni(spec, st[:, :2], st[:, 4:4 + 16, :2])
    np.testing.assert_allclose(c[0, 0, 1], 0.05 - 0.01 + 0.1, atol=1e-6)


def test_omni_dynamics_by_hand():
    spec = O.Spec("LidarOmniTarget", 1, 0)
    x = np.array([[[0.5, 0.5, 1.0, 0.0, 0.2, -0.1, 2.0]]], F)
    a = np.array([[[0.5, -1.0, 3.0]]], F)
    y = O.step_omni(spec, x, a)[0, 0]
    dt = 0.03
    np.testing.assert_allclose(y[:2], [0.5 + 0.2 * dt, 0.5 - 0.1 * dt], atol=1e-7)
    np.testing.assert_allclose(y[2:4], [np.cos(2.0 * dt), np.sin(2.0 * dt)], atol=1e-6)
    np.testing.assert_allclose(y[4:], [0.2 + 5 * dt, -0.1 - 10 * dt, 2.0 + 15 * dt], atol=1e-6)
    # velocity and angular-rate limits
    x = np.array([[[0.5, 0.5, 1.0, 0.0, 1.99, 0.0, 99.99]]], F)
    y = O.step_omni(spec, x, np.array([[[1.0, 0.0, 1.0]]], F))[0, 0]
    assert y[4] == F(2.0) and y[6] == F(100.0)


def test_omni_edge_features_local_frame():
    spec = O.Spec("LidarOmniTarget", 3, 0)
    ag = np.array([[[0.5, 0.5, 0.0, 1.0, 0, 0, 0],   # faces +y
                    [0.5, 0.7, 1.0, 0.0, 0, 0, 0],
                    [0.9, 0.7, 1.0, 0.0, 0, 0, 0]]], F)
    g = O.build_graph(spec, ag, np.zeros_like(ag), None)
    e = g["edges"][0]
    # edge (0 <- 1) is row 0*3 + 1: p_1 - p_0 = (0, 0.2); agent 0 faces +y -> local (0.2, 0)
    np.testing.assert_allclose(e[1, 7:], [1.0, 0.2, 0.2], atol=1e-6)  # critical, ||p||, forward
    np.testing.assert_allclose(e[3, 7], 0.0)  # (1 <- 0) is not critical
    np.testing.assert_allclose(e[5, 7:], [1.0, 0.4, 0.4], atol=1e-6)  # (1 <- 2): ahead of agent 1 along +x
    assert g["receivers"][0, 2] == 0  # (0, 2): |p| = 0.447 < comm_radius 0.5 -> kept
    assert g["receivers"][0, 0] == spec.n_nodes - 1  # self edge -> pad


def test_env_variant_goal_rules_kat():
    """landmark2goal by hand: LidarLine n=5 on (0,0)-(1,2) -> k/4 steps incl. both ends; MPELine n=3 ->
    the interior quarter points; MPEFormation n=4, R=0.5 around (1,1) -> (1.5,1), (1,1.5), (0.5,1), (1,0.5)."""
    from oracle import env_variants as V

    lm = np.array([[[0.0, 0.0], [1.0, 2.0]]], np.float32)
    g = V.landmark2goal(O.Spec("LidarLine", 5, 0), lm)[0]
    np.testing.assert_array_equal(g, np.array([[0, 0], [0.25, 0.5], [0.5, 1.0], [0.75, 1.5], [1, 2]], np.float32))
    g = V.landmark2goal(O.Spec("MPELine", 3, 0), lm)[0]
    np.testing.assert_array_equal(g, np.array([[0.25, 0.5], [0.5, 1.0], [0.75, 1.5]], np.float32))
    g = V.landmark2goal(O.Spec("MPEFormation", 4, 0), np.array([[[1.0, 1.0]]], np.float32))[0]
    np.testing.assert_allclose(g, [[1.5, 1.0], [1.0, 1.5], [0.5, 1.0], [1.0, 0.5]], atol=1e-6)
    # graph layout of the variants: goal node rows 2 / 1 / n
    for eid, n, ng in (("LidarLine", 5, 2), ("MPEFormation", 4, 1), ("MPECorridor", 3, 3)):
        spec = O.Spec(eid, n, 2)
        assert spec.ng == ng and (O.node_type(spec) == 1).sum() == ng

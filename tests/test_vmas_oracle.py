"""Known-answer tests of the VMAS restatement (oracle/vmas.py) against float64 forms of the reference's
formulas (env/vmas/physax/world.py, geometry.py, vmas_wheel.py, vmas_reverse_transport.py).  The reference
ships no VMAS fixtures and JAX is absent, so these pin the oracle (parity with the reference itself is
unpinned); tests/test_vmas_gpu.py then holds the HIP kernels bit-exact to it.  CPU only."""
import math

import numpy as np
import pytest

from oracle import math32
from oracle import vmas as V

F = np.float32


def test_logaddexp_twin_accuracy():
    x = np.linspace(-60, 60, 40001).astype(F)
    ref = np.logaddexp(0.0, x.astype(np.float64))
    assert np.max(np.abs(math32.logaddexp0(x) - ref) / np.maximum(np.abs(ref), 1e-30)) < 5e-7
    y = np.concatenate([np.linspace(0, 1, 20001), 10.0 ** np.arange(-30, 0)]).astype(F)
    ref = np.log1p(y.astype(np.float64))
    assert np.max(np.abs(math32.log1p(y) - ref) / np.maximum(ref, 1e-38)) < 5e-7
    assert math32.log1p(F(0)) == 0 and math32.exp_nonpos(F(-100)) == 0


@pytest.mark.parametrize("d", [0.0, 1e-7, 0.01, 0.03, 0.0366, 0.0367, 0.05])
def test_constraint_force_matches_float64(d):
    """world.py:440-468: f = mult * delta / |delta| * k * log(1 + exp((dmin - |delta|) / k)), zero when
    |delta| > dmin or < 1e-6."""
    dmin, k, mult = F(0.03 + 4 / 6e2), F(1e-3), F(100)
    ang = 0.7
    ax, ay = F(0.2 + d * math.cos(ang)), F(-0.1 + d * math.sin(ang))
    fx, fy = V.constraint_force(ax, ay, F(0.2), F(-0.1), dmin, mult, k)
    dd = math.hypot(float(ax) - 0.2, float(ay) + 0.1)
    if dd > float(dmin) or dd < 1e-6:
        assert fx == 0 and fy == 0
        return
    pen = float(k) * math.log1p(math.exp((float(dmin) - dd) / float(k)))
    ex, ey = 100 * (float(ax) - 0.2) / dd * pen, 100 * (float(ay) + 0.1) / dd * pen
    assert abs(fx - ex) <= 2e-5 * abs(ex) + 1e-9 and abs(fy - ey) <= 2e-5 * abs(ey) + 1e-9


def test_closest_point_line_and_box():
    # horizontal line of half-length 1 at the origin
    assert V.closest_point_line(F(0), F(0), F(1), F(0), F(1), F(0.5), F(0.3)) == (F(0.5), F(0))
    assert V.closest_point_line(F(0), F(0), F(1), F(0), F(1), F(-1.7), F(0.3)) == (F(-1), F(0))
    # box centred at (0.1, 0.2), sides 0.6: a point inside near the right wall -> on the right wall
    cx, cy = V.closest_point_box(F(0.1), F(0.2), F(0.3), F(0.37), F(0.25))
    assert abs(cx - 0.4) < 1e-6 and abs(cy - 0.25) < 1e-6
    # outside below the bottom wall
    cx, cy = V.closest_point_box(F(0.1), F(0.2), F(0.3), F(0.0), F(-0.2))
    assert abs(cx - 0.0) < 1e-6 and abs(cy - (-0.1)) < 1e-6


def test_free_motion_drag_and_integration():
    """No contact: v <- 0.75 v + F dt (world.py:107-135), x <- x + v dt, clipped to +-1.2."""
    st, rec = V.reset(V.WHEEL, 5, 1)
    st[0, :3, 0] = [1.19, -1.0, 0.9]
    st[0, :3, 1] = [1.15, 1.0, -0.9]  # far from the line through the origin at angle st[0,3,0]
    st[0, 3, :2] = [F(-math.pi / 4), F(0)]
    st[0, :3, 2:] = 0.1
    a = np.full((1, 3, 2), 0.5, F)
    out = V.step(V.WHEEL, st, rec, a)["states"][0]
    x, v = np.array(st[0, :3, :2], np.float64), np.array(st[0, :3, 2:], np.float64)
    for _ in range(3):
        v = v * 0.75 + 0.5 * 0.6 * 0.1
        x = np.clip(x + v * 0.1, -1.2, 1.2)
    np.testing.assert_allclose(out[:3, 2:], v, rtol=1e-5)
    np.testing.assert_allclose(out[:3, :2], x, rtol=1e-5, atol=1e-6)
    assert out[0, 0] == F(1.2)  # clipped at the world edge
    # the line (no torque): w <- 0.985 w per world step
    assert out[3, 1] == 0


def test_wheel_push_turns_the_line():
    """An agent pressed against the +x arm from below pushes it up: positive torque, counter-clockwise."""
    st, rec = V.reset(V.WHEEL, 5, 1)
    st[0, 3, :2] = [0, 0]
    st[0, 0] = [0.8, -0.02, 0, 0]
    st[0, 1] = [-1.1, 1.1, 0, 0]
    st[0, 2] = [1.1, 1.1, 0, 0]
    out = V.step(V.WHEEL, st, rec, np.zeros((1, 3, 2), F))
    assert out["states"][0, 3, 1] > 0 and out["states"][0, 3, 0] > 0
    s = dict(px=st[0, :3, 0].copy(), py=st[0, :3, 1].copy(), vx=np.zeros(3, F), vy=np.zeros(3, F),
             fx=np.zeros(3, F), fy=np.zeros(3, F), rot=F(0), w=F(0))
    fcx, fcy = V.wheel_world_step(s)  # first world step: the line pushes agent 0 down, the others are free
    assert fcy[0] < 0 and abs(fcx[0]) < 1e-6 and (fcx[1:] == 0).all() and (fcy[1:] == 0).all()
    # angular velocity is clamped at 0.6 (clamp_with_norm, vmas_utils.py:6-10)
    st[0, 3, 1] = 2.0
    out = V.step(V.WHEEL, st, rec, np.zeros((1, 3, 2), F))
    assert abs(out["states"][0, 3, 1]) <= F(0.6)


def test_transport_box_pushed_by_agents():
    st, rec = V.reset(V.TRANSPORT, 3, 1)
    bx, by = st[0, 3, 0], st[0, 3, 1]
    st[0, :3, 0] = bx + np.array([0.28, 0.0, -0.1], F)  # agent 0 against the inside of the right wall
    st[0, :3, 1] = by + np.array([0.0, 0.05, -0.05], F)
    st[0, :3, 2:] = 0
    st[0, 3, 2:] = 0
    a = np.zeros((1, 3, 2), F)
    a[0, 0, 0] = 1.0  # pushes right
    out = V.step(V.TRANSPORT, st, rec, a)["states"][0]
    assert out[3, 2] > 0 and out[3, 0] > bx and abs(out[3, 3]) < 1e-6


@pytest.mark.parametrize("kind", [V.WHEEL, V.TRANSPORT])
def test_reset_invariants(kind):
    st, rec = V.reset(kind, 17, 64)
    p = st[:, :3, :2].astype(np.float64)
    d = np.linalg.norm(p[:, :, None] - p[:, None], axis=-1) + np.eye(3) * 10
    assert (d > 0.06).all()  # get_node_goal_rng min_dist 2 r
    assert (np.abs(st[:, :3, 2:]) <= 0.01).all()
    if kind == V.WHEEL:
        assert (np.abs(p) <= 1.2).all() and (np.abs(st[:, 3, 0]) <= np.pi + 1e-6).all()
        assert (np.abs(st[:, 3, 1]) <= 0.05).all()
        ok = 0
        for b in range(64):  # sample_valid_avoid_angle: valid when any of the 8 draws was
            dg = abs(V.angle_dist(rec[b, 0, 1], rec[b, 0, 0]))
            dl = abs(V.angle_dist(rec[b, 0, 1], st[b, 3, 0]))
            ok += int(dg > V.W["avoid_min"] and dl > V.W["avoid_min"] and dg < V.W["goal_max"])
        assert ok >= 56
    else:
        box = st[:, 3, :2].astype(np.float64)
        assert np.allclose(np.linalg.norm(box, axis=-1), 0.49, atol=1e-6)
        goal = rec[:, 0, :2].astype(np.float64)
        assert np.allclose(np.linalg.norm(goal, axis=-1), 0.49, atol=1e-6)
        cosang = (box * goal).sum(-1) / (0.49 * 0.49)
        assert (cosang <= -math.cos(math.radians(30)) + 1e-5).all()  # goal opposite, +-30 deg
        o = rec[:, 0, 2:].reshape(-1, 3, 2).astype(np.float64)
        assert np.allclose(np.linalg.norm(o, axis=-1), 0.49 - 0.225, atol=1e-6)
        assert (np.abs(p - box[:, None]) <= 0.2 + 1e-6).all()
        assert (st[:, 3, 2:] == 0).all()


@pytest.mark.parametrize("kind", [V.WHEEL, V.TRANSPORT])
def test_graph_layout_and_cost_ranges(kind):
    st, rec = V.reset(kind, 23, 8)
    g = V.initial_graph(kind, st, rec)
    assert g["nodes"].shape == (8, 4, V.NODE_DIM[kind]) and (g["nodes"][:, 3] == 0).all()
    assert (g["receivers"][0] == [3, 0, 0, 1, 3, 1, 2, 2, 3]).all()
    assert (g["senders"][0] == [3, 1, 2, 0, 3, 2, 0, 1, 3]).all()
    np.testing.assert_array_equal(g["edges"][:, 1], st[:, 0] - st[:, 1])
    a = np.random.default_rng(0).uniform(-1, 1, (8, 3, 2)).astype(F)
    out = V.step(kind, st, rec, a)
    c = out["cost"]
    assert (c >= -1).all() and ((np.abs(c) >= 0.5) | (c == -1)).all()  # the +-0.5 margin
    if kind == V.TRANSPORT:
        assert (c <= 1).all()
        n = g["nodes"]
        assert (np.diff(n[:, :3, 17:20], axis=-1) >= 0).all()  # obstacle distances sorted
        np.testing.assert_allclose(np.linalg.norm(n[:, :3, 11:17].reshape(8, 3, 3, 2), axis=-1), 1, atol=1e-5)
    else:
        n = g["nodes"]
        np.testing.assert_allclose(n[:, :3, 4] ** 2 + n[:, :3, 5] ** 2, 1, atol=1e-6)
        assert (n[:, :3, 7:9] == 0).all()  # reset: no contact force yet
    assert out["reward"].shape == (8,) and (out["reward"] <= 0).all()

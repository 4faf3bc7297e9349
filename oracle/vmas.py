"""NumPy fp32 restatement of the reference's VMAS environments (VMASWheel, VMASReverseTransport) and the
contact-physics world they step (TEST INFRASTRUCTURE ONLY, see oracle/__init__.py; parity unpinned: the
reference ships no VMAS fixtures and JAX is absent, so the restatement is checked by its own known-answer
tests in tests/test_vmas_oracle.py and the HIP kernels are checked against it bit for bit).

Reference:
  env/vmas/vmas_wheel.py:90-122 (reset), :124-216 (step), :218-260 (reward, cost), :262-307 (graph),
      :425-452 (angle_dist, sample_valid_avoid_angle)
  env/vmas/vmas_reverse_transport.py:91-129 (reset), :131-207 (step), :209-250 (reward, cost),
      :252-312 (in-contact test, graph)
  env/vmas/physax/world.py:78-105 (World.step), :107-163 (integration), :193-268 (contact pairs),
      :309-359 (sphere-line), :361-438 (box-sphere), :440-468 (_get_constraint_forces), :579-589
  env/vmas/physax/geometry.py:8-34 (closest point on a line), :37-102 (box sides)
  env/vmas/physax/vmas_utils.py:6-10 (clamp_with_norm), :31-36 (cross / torque)
  env/utils.py:139-244 (get_node_goal_rng; oracle/env.py:node_goal_rng)

Layout of the framework's VMAS graphs (the reference pads GetGraph states to width 0; these carry the
env state instead, in the same (B, N=4, 4) `states` tensor every other env uses):
  states rows 0..2  agent [x, y, vx, vy]
  states row 3      Wheel [line_angle, line_angvel, 0, 0] / Transport [box_x, box_y, box_vx, box_vy]
  record (B, 1, 8)  Wheel [goal_angle, avoid_angle, 0 x 6] / Transport [goal_x, goal_y, o0x, o0y, .., o2y]
Every expression is evaluated as the reference does with jax_enable_x64 off: Python-float constants are
rounded once to fp32 (double arithmetic first, e.g. 1 - drag), every op rounds once, in the reference's order.
jax.random is replaced by Philox streams, one per jax.random.split key (purpose = split index + 1).
"""
from __future__ import annotations

import numpy as np

from . import math32
from .env import node_goal_rng

F = np.float32
WHEEL, TRANSPORT = "VMASWheel", "VMASReverseTransport"
N_AGENTS, N_NODES, N_EDGES, SD, REC = 3, 4, 9, 4, 8
NODE_DIM = {WHEEL: 13, TRANSPORT: 20}
PI = np.pi

# ---- constants (python float64 expressions, rounded once) ------------------------------------------------
LINE_MIN_DIST = 4 / 6e2                       # world.py:19
AGENT_R = 0.03
# VMASWheel (vmas_wheel.py:53-64, 132-164; world.py defaults: dt 0.1, substeps 1, margin 1e-3, force 100)
W = dict(u_mult=F(0.6), agent_drag=F(1 - 0.25), line_drag=F(1 - 0.015), sub_dt=F(0.1 / 1),
         moi=F((1 / 12) * 15.0 * (2.0 ** 2)), max_w=F(0.6), dmin=F(AGENT_R + LINE_MIN_DIST), k=F(1e-3),
         mult=F(100), semi=F(1.2), half_len=F(2.0 / 2), side=0.99 * (2 * 1.2), shift=F(1.2),
         obs_hw=F(np.deg2rad(15)), avoid_min=F(np.deg2rad(15) + np.deg2rad(1)), goal_max=F(np.pi / 2),
         rew_deg=F(np.deg2rad(1)), frame_skip=3, substeps=1)
# VMASReverseTransport (vmas_reverse_transport.py:50-64, 139-161; World(contact_margin=6e-3, substeps=5,
# collision_force=500))
_X0R = 0.98 * (0.8 - 0.5 * 0.6)
T_ = dict(u_mult=F(0.5), agent_drag=F(1 - 0.25), box_drag=F(1 - 0.25), sub_dt=F(0.1 / 5), box_mass=F(10.0),
          dmin=F(AGENT_R + LINE_MIN_DIST), k=F(6e-3), mult=F(500), semi=F(1.2), half=F(0.6 / 2),
          side=0.4 * 0.6, shift=F(0.2), x0r=F(_X0R), obs_place_r=F(_X0R - 1.5 * 0.15), noise_ub=np.deg2rad(30),
          obs_r=F(0.15), contact_len=F(0.6 - 1e-2), dist2goal=F(0.01), frame_skip=4, substeps=5)
AGENT_COST = F(AGENT_R * 2)


class Stream:
    """One jax.random key: Philox counter (draw, env, purpose, 0) keyed by the reset seed."""

    def __init__(self, seed, env, purpose):
        self.k0, self.k1 = seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF
        self.env, self.purpose, self.count = int(env), int(purpose), 0

    def uniform(self, lo, hi):
        bits = math32.philox4x32(self.count, self.env, self.purpose, 0, self.k0, self.k1)[0]
        self.count += 1
        return F(math32.uniform(bits, lo, hi))


def angle_dist(a, b):
    """vmas_wheel.py:425-427: atan2(sin(a - b), cos(a - b))."""
    s, c = math32.sincos(F(a) - F(b))
    return math32.atan2(s, c)


def _norm(dx, dy):
    return np.sqrt(F(dx) * F(dx) + F(dy) * F(dy)).astype(F)


# ---- physics (world.py) -------------------------------------------------------------------------------
def constraint_force(ax, ay, bx, by, dmin, mult, k):
    """_get_constraint_forces (world.py:440-468), not attractive: the force on a (b gets its negative)."""
    dx, dy = F(ax) - F(bx), F(ay) - F(by)
    d = _norm(dx, dy)
    pen = math32.logaddexp0(((dmin - d) * F(1)) / k) * k
    den = d if d > 0 else F(1e-8)
    fx, fy = ((mult * dx) / den) * pen, ((mult * dy) / den) * pen
    if d < F(1e-6) or d > dmin:
        return F(0), F(0)
    return F(fx), F(fy)


def closest_point_line(lx, ly, rvx, rvy, half_len, px, py):
    """geometry.py:8-34 with the line direction (cos rot, sin rot) precomputed."""
    dx, dy = F(lx) - F(px), F(ly) - F(py)
    dot = dx * rvx + dy * rvy
    sg = F(np.sign(dot))
    dfc = min(abs(dot), half_len)
    s = sg * dfc
    return F(lx - s * rvx), F(ly - s * rvy)


def _box_lines(bx, by, half):
    """get_all_lines_box (geometry.py:78-102) for box_rot = 0: side midpoints and directions."""
    s0, c0 = math32.sincos(F(0))
    rot2 = F(0) + F(np.pi / 2)
    s2, c2 = math32.sincos(rot2)
    rv, rv2 = (F(c0), F(s0)), (F(c2), F(s2))
    p1 = (bx + rv[0] * half, by + rv[1] * half)
    p2 = (bx - rv[0] * half, by - rv[1] * half)
    p3 = (bx + rv2[0] * half, by + rv2[1] * half)
    p4 = (bx - rv2[0] * half, by - rv2[1] * half)
    # lines 0, 1 rotate by box_rot + pi/2, lines 2, 3 by box_rot; every side is 0.6 long
    return [(p1, rv2), (p2, rv2), (p3, rv), (p4, rv)]


def closest_point_box(bx, by, half, px, py):
    """get_closest_point_box (geometry.py:37-53): the first side midpoint-line point of minimal distance."""
    best, dist = (F(np.inf), F(np.inf)), F(np.inf)
    for (lx, ly), (rvx, rvy) in _box_lines(bx, by, half):
        c = closest_point_line(lx, ly, rvx, rvy, half, px, py)
        d = _norm(px - c[0], py - c[1])
        if d < dist:
            best, dist = c, d
    return best


def wheel_world_step(s):
    """One World.step (world.py:78-105) of the wheel scene [line, agent_0..2]; s is a dict of fp32 scalars /
    arrays (px, py, vx, vy (3,), fx, fy (3,) action forces, rot, w).  Returns the agents' contact forces."""
    K = W
    c_s, c_c = math32.sincos(s["rot"])
    rvx, rvy = F(c_c), F(c_s)
    torque = None
    fcx, fcy = np.zeros(3, F), np.zeros(3, F)
    for i in range(3):  # pairs (line, agent_i), world.py:309-359
        cx, cy = closest_point_line(F(0), F(0), rvx, rvy, K["half_len"], s["px"][i], s["py"][i])
        fx, fy = constraint_force(s["px"][i], s["py"][i], cx, cy, K["dmin"], K["mult"], K["k"])
        flx, fly = -fx, -fy
        rx, ry = F(cx - F(0)), F(cy - F(0))
        t = F(rx * fly - ry * flx)
        torque = t if torque is None else F(torque + t)
        fcx[i], fcy[i] = fx, fy
    tq = F(F(0) + torque)
    Fx = (F(0) + s["fx"]) + fcx
    Fy = (F(0) + s["fy"]) + fcy
    # line: not movable, rotatable (world.py:137-152)
    w = s["w"] * K["line_drag"]
    w = F(w + (tq / K["moi"]) * K["sub_dt"])
    nrm = F(np.sqrt(w * w))
    if nrm > K["max_w"]:
        w = F((w / nrm) * K["max_w"])
    s["rot"] = F(s["rot"] + w * K["sub_dt"])
    s["w"] = w
    _integrate_agents(s, Fx, Fy, K["agent_drag"], K["sub_dt"], K["semi"], True)
    return fcx, fcy


def _integrate_agents(s, Fx, Fy, drag, dt, semi, substep0):
    vx, vy = s["vx"], s["vy"]
    if substep0:
        vx, vy = (vx * drag).astype(F), (vy * drag).astype(F)
    vx = (vx + (Fx / F(1.0)) * dt).astype(F)
    vy = (vy + (Fy / F(1.0)) * dt).astype(F)
    s["vx"], s["vy"] = vx, vy
    s["px"] = np.minimum(np.maximum((s["px"] + vx * dt).astype(F), -semi), semi).astype(F)
    s["py"] = np.minimum(np.maximum((s["py"] + vy * dt).astype(F), -semi), semi).astype(F)


def transport_world_step(s):
    """One World.step of the transport scene [box, agent_0..2] (5 substeps)."""
    K = T_
    for sub in range(K["substeps"]):
        fcx, fcy = np.zeros(3, F), np.zeros(3, F)
        fb = None
        for i in range(3):  # pairs (box, agent_i), world.py:361-438
            cx, cy = closest_point_box(s["bx"], s["by"], K["half"], s["px"][i], s["py"][i])
            fx, fy = constraint_force(s["px"][i], s["py"][i], cx, cy, K["dmin"], K["mult"], K["k"])
            fcx[i], fcy[i] = fx, fy
            fb = (-fx, -fy) if fb is None else (F(fb[0] + -fx), F(fb[1] + -fy))
        Fbx, Fby = F(F(0) + fb[0]), F(F(0) + fb[1])
        Fx = (F(0) + s["fx"]) + fcx
        Fy = (F(0) + s["fy"]) + fcy
        # box: movable, not rotatable (world.py:107-135)
        bvx, bvy = s["bvx"], s["bvy"]
        if sub == 0:
            bvx, bvy = F(bvx * K["box_drag"]), F(bvy * K["box_drag"])
        bvx = F(bvx + (Fbx / K["box_mass"]) * K["sub_dt"])
        bvy = F(bvy + (Fby / K["box_mass"]) * K["sub_dt"])
        s["bvx"], s["bvy"] = bvx, bvy
        s["bx"] = F(min(max(F(s["bx"] + bvx * K["sub_dt"]), -K["semi"]), K["semi"]))
        s["by"] = F(min(max(F(s["by"] + bvy * K["sub_dt"]), -K["semi"]), K["semi"]))
        _integrate_agents(s, Fx, Fy, K["agent_drag"], K["sub_dt"], K["semi"], sub == 0)


# ---- reward / cost (on the pre-step state) ------------------------------------------------------------
def _agent_min_dist(px, py):
    md = np.zeros(3, F)
    for i in range(3):
        ds = [F(_norm(px[i] - px[j], py[i] - py[j]) + (F(1e6) if i == j else F(0))) for j in range(3)]
        md[i] = min(ds)
    return md


def _margin(c, lo, hi):
    c = np.where(c <= 0, c - F(0.5), c + F(0.5)).astype(F)
    c = np.maximum(c, F(lo))
    return (np.minimum(c, F(hi)) if hi is not None else c).astype(F)


def wheel_reward_cost(st, rec):
    line = st[3, 0]
    ad = angle_dist(line, rec[0, 0])
    sq = F(F(F(0.1) * ad) / F(PI))
    sq = F(sq * sq)
    r = F(F(-sq) * F(0.5))
    r = F(r - F(F(1.0 if ad > W["rew_deg"] else 0.0) * F(0.005)))
    md = _agent_min_dist(st[:3, 0], st[:3, 1])
    c_agent = (AGENT_COST - md).astype(F)
    ld = angle_dist(line, rec[0, 1])
    cl = F(F(W["obs_hw"] - abs(ld)) / F(PI))
    cost = np.stack([c_agent, np.full(3, cl, F)], -1)
    return r, _margin(cost, -1.0, None)


def transport_reward_cost(st, rec):
    bx, by = st[3, 0], st[3, 1]
    d = _norm(rec[0, 0] - bx, rec[0, 1] - by)
    r = F(F(-d) * F(0.01))
    r = F(r - F(F(1.0 if d > T_["dist2goal"] else 0.0) * F(0.001)))
    md = _agent_min_dist(st[:3, 0], st[:3, 1])
    a_cost = (AGENT_COST - md).astype(F)
    od = [_norm(bx - rec[0, 2 + 2 * o], by - rec[0, 3 + 2 * o]) for o in range(3)]
    cb = F(T_["obs_r"] - min(od))
    cost = np.stack([(F(4) * a_cost).astype(F), np.full(3, F(F(2) * cb), F)], -1)
    return r, _margin(cost, -1.0, 1.0)


# ---- graph (get_graph + edge_blocks + to_padded) -----------------------------------------------------
def build_graph(kind, st, rec, contact=None):
    """st (4, 4) states, rec (1, 8); contact (3, 2) the Wheel agents' last contact forces."""
    nd = NODE_DIM[kind]
    nodes = np.zeros((N_NODES, nd), F)
    nodes[:3, :4] = st[:3]
    if kind == WHEEL:
        line = st[3, 0]
        s, c = math32.sincos(line)
        nodes[:3, 4], nodes[:3, 5], nodes[:3, 6] = s, c, st[3, 1]
        if contact is not None:
            nodes[:3, 7:9] = contact
        for col, ang in ((9, rec[0, 0]), (11, rec[0, 1])):
            s, c = math32.sincos(angle_dist(line, ang))
            nodes[:3, col], nodes[:3, col + 1] = s, c
    else:
        bx, by = st[3, 0], st[3, 1]
        nodes[:3, 4:8] = st[3]
        nodes[:3, 8], nodes[:3, 9] = F(rec[0, 0] - bx), F(rec[0, 1] - by)
        rx, ry = (st[:3, 0] - bx).astype(F), (st[:3, 1] - by).astype(F)
        nodes[:3, 10] = ((np.abs(rx) > T_["contact_len"]) | (np.abs(ry) > T_["contact_len"])).astype(F)
        ox = np.array([F(rec[0, 2 + 2 * o] - bx) for o in range(3)], F)
        oy = np.array([F(rec[0, 3 + 2 * o] - by) for o in range(3)], F)
        od = np.sqrt((ox * ox + oy * oy) + F(1e-6)).astype(F)
        vx, vy = (ox / od).astype(F), (oy / od).astype(F)
        order = np.argsort(od, kind="stable")
        for q, o in enumerate(order):
            nodes[:3, 11 + 2 * q], nodes[:3, 12 + 2 * q], nodes[:3, 17 + q] = vx[o], vy[o], od[o]
    states = st.astype(F).copy()
    edges = np.zeros((N_EDGES, 4), F)
    recv = np.zeros(N_EDGES, np.int32)
    send = np.zeros(N_EDGES, np.int32)
    for i in range(3):
        for j in range(3):
            e = i * 3 + j
            edges[e] = st[i] - st[j]
            recv[e], send[e] = (i, j) if i != j else (3, 3)
    return dict(nodes=nodes, edges=edges, states=states, receivers=recv, senders=send)


# ---- reset / step (batched over envs) -------------------------------------------------------------------
def sample_valid_avoid_angle(stream, line, goal):
    """vmas_wheel.py:435-452."""
    b = np.array([stream.uniform(-PI, PI) for _ in range(8)], F)
    dg = np.abs(angle_dist(b, goal))
    dl = np.abs(angle_dist(b, line))
    ok = (dg > W["avoid_min"]) & (dl > W["avoid_min"]) & (dg < W["goal_max"])
    masked = np.where(ok, dg, F(np.inf))
    return b[int(np.argmin(masked))]


def reset(kind, seed, n_env, env_offset=0):
    """Returns (states (B,4,4), record (B,1,8))."""
    st = np.zeros((n_env, N_NODES, SD), F)
    rec = np.zeros((n_env, 1, REC), F)
    for b in range(n_env):
        e = env_offset + b
        S = lambda p: Stream(seed, e, p)  # noqa: E731
        if kind == WHEEL:
            line = S(1).uniform(-PI, PI)
            w = S(2).uniform(-0.05, 0.05)
            ap, _ = node_goal_rng(S(3), W["side"], 3, 2 * AGENT_R, None)
            sv = S(4)
            av = np.array([sv.uniform(-0.01, 0.01) for _ in range(6)], F).reshape(3, 2)
            goal = S(5).uniform(-PI, PI)
            avoid = sample_valid_avoid_angle(S(6), line, goal)
            st[b, :3, :2] = (ap - W["shift"]).astype(F)
            st[b, :3, 2:] = av
            st[b, 3, :2] = line, w
            rec[b, 0, :2] = goal, avoid
        else:
            x0 = S(1).uniform(0.0, 2 * PI)
            s0, c0 = math32.sincos(x0)
            box = (T_["x0r"] * F(c0), T_["x0r"] * F(s0))
            ga = F(F(x0 + F(PI)) + S(4).uniform(-T_["noise_ub"], T_["noise_ub"]))
            sg, cg = math32.sincos(ga)
            so = S(5)
            oa = np.array([so.uniform(0.0, 2 * PI) for _ in range(3)], F)
            sa, ca = math32.sincos(oa)
            ap, _ = node_goal_rng(S(2), T_["side"], 3, 2 * AGENT_R, None)
            sv = S(3)
            av = np.array([sv.uniform(-0.01, 0.01) for _ in range(6)], F).reshape(3, 2)
            st[b, :3, 0] = ((ap[:, 0] - T_["shift"]).astype(F) + F(box[0])).astype(F)
            st[b, :3, 1] = ((ap[:, 1] - T_["shift"]).astype(F) + F(box[1])).astype(F)
            st[b, :3, 2:] = av
            st[b, 3, :2] = box
            rec[b, 0, 0], rec[b, 0, 1] = T_["x0r"] * F(cg), T_["x0r"] * F(sg)
            rec[b, 0, 2::2] = (T_["obs_place_r"] * ca).astype(F)
            rec[b, 0, 3::2] = (T_["obs_place_r"] * sa).astype(F)
    return st, rec


def initial_graph(kind, st, rec):
    gs = [build_graph(kind, st[b], rec[b], np.zeros((3, 2), F) if kind == WHEEL else None) for b in range(len(st))]
    return {k: np.stack([g[k] for g in gs]) for k in gs[0]}


def step(kind, st, rec, action):
    """Batched env.step: st (B,4,4) pre-step states, rec (B,1,8), action (B,3,2).  Returns the next graph
    (dict) plus reward (B,), cost (B,3,2) of the pre-step state."""
    B = st.shape[0]
    out = {k: [] for k in ("nodes", "edges", "states", "receivers", "senders")}
    rew = np.zeros(B, F)
    cost = np.zeros((B, 3, 2), F)
    K = W if kind == WHEEL else T_
    for b in range(B):
        a = np.minimum(np.maximum(action[b].astype(F), F(-1)), F(1)).astype(F)
        if kind == WHEEL:
            rew[b], cost[b] = wheel_reward_cost(st[b], rec[b])
        else:
            rew[b], cost[b] = transport_reward_cost(st[b], rec[b])
        s = dict(px=st[b, :3, 0].copy(), py=st[b, :3, 1].copy(), vx=st[b, :3, 2].copy(), vy=st[b, :3, 3].copy(),
                 fx=(a[:, 0] * K["u_mult"]).astype(F), fy=(a[:, 1] * K["u_mult"]).astype(F))
        contact = None
        if kind == WHEEL:
            s.update(rot=st[b, 3, 0], w=st[b, 3, 1])
            for _ in range(K["frame_skip"]):
                fcx, fcy = wheel_world_step(s)
            contact = np.stack([fcx, fcy], -1)
            body = (s["rot"], s["w"], F(0), F(0))
        else:
            s.update(bx=st[b, 3, 0], by=st[b, 3, 1], bvx=st[b, 3, 2], bvy=st[b, 3, 3])
            for _ in range(K["frame_skip"]):
                transport_world_step(s)
            body = (s["bx"], s["by"], s["bvx"], s["bvy"])
        nst = np.zeros((N_NODES, SD), F)
        nst[:3] = np.stack([s["px"], s["py"], s["vx"], s["vy"]], -1)
        nst[3] = body
        g = build_graph(kind, nst, rec[b], contact)
        for k in out:
            out[k].append(g[k])
    res = {k: np.stack(v) for k, v in out.items()}
    res.update(reward=rew, cost=cost)
    return res


def rollout(kind, st, rec, actions):
    """T steps with actions (T, B, 3, 2): lists of graphs, rewards (T, B), costs (T, B, 3, 2)."""
    graphs, rews, costs = [], [], []
    for t in range(actions.shape[0]):
        g = step(kind, st, rec, actions[t])
        graphs.append(g)
        rews.append(g["reward"])
        costs.append(g["cost"])
        st = g["states"]
    return graphs, np.stack(rews), np.stack(costs)

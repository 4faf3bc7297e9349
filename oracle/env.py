"""NumPy restatement of the reference environment step / reset / graph build (hot path 1).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py — parity unpinned, no reference goldens exist).

Everything is batched over a leading env axis B and computed in float32 with one rounding per
operation, in the reference's operation order, so that the HIP kernels (compiled with
-ffp-contract=off) reproduce it bit for bit.  Reductions that only feed continuous outputs (the
reward means) are summed sequentially over agents — the reference leaves that order to XLA.
"""
from __future__ import annotations

import dataclasses
import math

import numpy as np

from . import math32

F = np.float32

# ---- reference PARAMS dicts (class attributes) ---------------------------------------------
LIDAR_PARAMS = {  # lidar_env/base.py:41-50, lidar_spread.py:13-22, lidar_target.py:13-22, bicycle:24-33
    "car_radius": 0.05, "comm_radius": 0.5, "n_rays": 32, "obs_len_range": [0.1, 0.3], "n_obs": 3,
    "default_area_size": 1.5, "dist2goal": 0.01, "top_k_rays": 8,
}
MPE_PARAMS = {  # mpe_spread.py:12-19, mpe_target.py:12-19
    "car_radius": 0.05, "comm_radius": 0.5, "n_obs": 3, "obs_radius": 0.05, "default_area_size": 1.5,
    "dist2goal": 0.01,
}

OMNI_PARAMS = dict(LIDAR_PARAMS, **{  # lidar_omni_target.py:49-68
    "max_angular_vel": 100.0, "rotation_penalty": 0.001, "fov_angle_deg": 60.0, "max_sensor_range": 0.5,
    "min_safe_distance": 0.2,
})

ENGINE_LIDAR, ENGINE_BICYCLE, ENGINE_MPE, ENGINE_OMNI = 0, 1, 2, 3
GOAL_SPREAD, GOAL_TARGET = 0, 1
# reference env variants (oracle/env_variants.py): goal-node layout, reward goals, resets, costs
VARIANT_NONE, VARIANT_LINE, VARIANT_FORMATION, VARIANT_CORRIDOR, VARIANT_CONNECT = 0, 1, 2, 3, 4
MPE_CORRIDOR_PARAMS = {  # mpe_corridor.py:14-21 (obs_radius derived in __init__, :37)
    "car_radius": 0.05, "comm_radius": 0.5, "default_area_size": 1.0, "dist2goal": 0.01, "n_obs": 2,
    "corridor_width": 0.2,
}
MPE_CONNECT_PARAMS = {  # mpe_connect_spread.py:16-24
    "car_radius": 0.05, "comm_radius": 0.5, "default_area_size": 1.0, "dist2goal": 0.01, "n_obs": 1,
    "obs_radius": 0.25, "connect_radius": 0.45,
}

ENVS = {
    "LidarSpread": (ENGINE_LIDAR, GOAL_SPREAD),
    "LidarTarget": (ENGINE_LIDAR, GOAL_TARGET),
    "LidarBicycleTarget": (ENGINE_BICYCLE, GOAL_TARGET),
    "MPESpread": (ENGINE_MPE, GOAL_SPREAD),
    "MPETarget": (ENGINE_MPE, GOAL_TARGET),
    "LidarOmniTarget": (ENGINE_OMNI, GOAL_TARGET),
    "LidarLine": (ENGINE_LIDAR, GOAL_SPREAD),  # lidar_line.py (LidarSpread params, 2 landmark goal nodes)
    "MPELine": (ENGINE_MPE, GOAL_SPREAD),  # mpe_line.py (MPESpread params)
    "MPEFormation": (ENGINE_MPE, GOAL_SPREAD),  # mpe_formation.py
    "MPECorridor": (ENGINE_MPE, GOAL_SPREAD),  # mpe_corridor.py
    "MPEConnectSpread": (ENGINE_MPE, GOAL_SPREAD),  # mpe_connect_spread.py
}
VARIANTS = {"LidarLine": VARIANT_LINE, "MPELine": VARIANT_LINE, "MPEFormation": VARIANT_FORMATION,
            "MPECorridor": VARIANT_CORRIDOR, "MPEConnectSpread": VARIANT_CONNECT}


@dataclasses.dataclass
class Spec:
    env_id: str
    n: int
    n_obs: int
    n_rays: int = 32
    top_k: int = 8
    dt: float = 0.03
    full_observation: bool = False

    def __post_init__(self):
        self.engine, self.goal_mode = ENVS[self.env_id]
        self.variant = VARIANTS.get(self.env_id, VARIANT_NONE)
        p = dict(MPE_PARAMS if self.engine == ENGINE_MPE else (OMNI_PARAMS if self.engine == ENGINE_OMNI else LIDAR_PARAMS))
        if self.variant == VARIANT_CORRIDOR:
            p = dict(MPE_CORRIDOR_PARAMS)
            p["obs_radius"] = (p["default_area_size"] - p["corridor_width"]) / 4  # mpe_corridor.py:37
            self.n_obs = 2  # forced (mpe_corridor.py:33-35)
        elif self.variant == VARIANT_CONNECT:
            p = dict(MPE_CONNECT_PARAMS)
            self.n_obs = 1  # forced (mpe_connect_spread.py:38-40)
        self.params = p
        self.car_r = p["car_radius"]
        self.comm_r = p["comm_radius"]
        self.area = p["default_area_size"]
        if self.full_observation:  # env/__init__.py:46-48
            self.comm_r = self.area * 10
        self.obs_r = p.get("obs_radius", 0.0)
        self.dist2goal = p["dist2goal"]
        self.obs_len_range = p.get("obs_len_range", [0.1, 0.3])
        self.sd = {ENGINE_BICYCLE: 5, ENGINE_OMNI: 7}.get(self.engine, 4)
        self.nd = self.sd + 3
        omni = self.engine == ENGINE_OMNI
        self.ed = 10 if omni else 4  # edge_dim (lidar_omni_target.py:136-143)
        self.ad = 3 if omni else 2  # action_dim (ax, ay, alpha)
        self.n_cost = 5 if omni else (3 if self.variant == VARIANT_CONNECT else 2)
        # goal node rows: 2 landmarks (line), 1 landmark (formation), else one per agent
        self.ng = {VARIANT_LINE: 2, VARIANT_FORMATION: 1}.get(self.variant, self.n)

    @property
    def has_lidar(self):
        return self.engine != ENGINE_MPE and self.n_obs > 0

    @property
    def n_hits(self):
        return self.n * self.top_k if self.has_lidar else 0

    @property
    def n_nodes(self):  # graph.py:212-247 (+1 pad node)
        if self.engine == ENGINE_MPE:
            return self.n + self.ng + self.n_obs + 1
        return self.n + self.ng + self.n_hits + 1

    @property
    def n_ag(self):
        return self.n * self.ng if self.goal_mode == GOAL_SPREAD else self.n

    @property
    def n_edges(self):
        if self.engine == ENGINE_MPE:
            return self.n * self.n + self.n_ag + self.n * self.n_obs
        return self.n * self.n + self.n_ag + self.n_hits

    def state_lim(self):
        if self.engine == ENGINE_OMNI:  # lidar_omni_target.py:502-509
            w = self.params["max_angular_vel"]
            return (np.array([0, 0, -1, -1, -2, -2, -w], F), np.array([self.area, self.area, 1, 1, 2, 2, w], F))
        if self.engine == ENGINE_BICYCLE:  # lidar_bicycle_target.py:120-123
            return (np.array([0, 0, -1, -1, -0.5], F), np.array([self.area, self.area, 1, 1, 0.5], F))
        if self.engine == ENGINE_MPE:  # mpe/base.py:243-246; corridor / connect: y up to 2 area
            hy = 2 * self.area if self.variant in (VARIANT_CORRIDOR, VARIANT_CONNECT) else self.area
            return np.array([0, 0, -1, -1], F), np.array([self.area, hy, 1, 1], F)
        return np.array([0, 0, -0.5, -0.5], F), np.array([self.area, self.area, 0.5, 0.5], F)  # lidar base 273-276


# ---- NaN-propagating helpers (jnp.minimum / jnp.clip semantics) ------------------------------
def clip(x, lo, hi):
    """jnp.clip = minimum(maximum(x, lo), hi), NaN-propagating."""
    return np.minimum(np.maximum(x, lo), hi).astype(F)


def norm2d(dx, dy):
    """jnp.linalg.norm over a 2-vector: sqrt(dx*dx + dy*dy)."""
    return np.sqrt(dx * dx + dy * dy).astype(F)


# ---- geometry ------------------------------------------------------------------------------
def ray_thetas(n_rays: int):
    """jnp.linspace(-pi, pi - 2pi/R, R) in float32 (env/utils.py:51), JAX's start*(1-s)+stop*s form."""
    start = F(-np.pi)
    stop = F(np.pi - 2 * np.pi / n_rays)
    if n_rays == 1:
        return np.array([start], F)
    div = n_rays - 1
    step = (np.arange(div, dtype=F) / F(div)).astype(F)
    out = start * (F(1) - step) + stop * step
    return np.concatenate([out, [stop]]).astype(F)


def ray_table(n_rays: int, sense_range: float):
    """(R, 2): (cos th * range, sin th * range) — the per-ray end offsets of env/utils.py:53-55."""
    s, c = math32.sincos(ray_thetas(n_rays))
    r = F(sense_range)
    return np.stack([c * r, s * r], axis=-1).astype(F)


OBST_FIELDS = 16  # [cx, cy, w, h, theta, cos, sin, type, p0x, p0y, p1x, p1y, p2x, p2y, p3x, p3y]


def make_rectangles(center, width, height, theta):
    """Rectangle.create (env/obstacle.py:39-56), packed into 16-float records.

    Fields 5,6 cache cos/sin(theta) (the reference recomputes them inside `inside()`)."""
    center = np.asarray(center, F)
    w = np.asarray(width, F)
    h = np.asarray(height, F)
    th = np.asarray(theta, F)
    s, c = math32.sincos(th)
    hw, hh = w / F(2), h / F(2)
    bx = np.stack([hw, -hw, -hw, hw], axis=-1)
    by = np.stack([hh, hh, -hh, -hh], axis=-1)
    c4, s4 = c[..., None], s[..., None]
    px = (c4 * bx + (-s4) * by) + center[..., 0:1]
    py = (s4 * bx + c4 * by) + center[..., 1:2]
    rec = np.zeros(center.shape[:-1] + (OBST_FIELDS,), F)
    rec[..., 0:2] = center
    rec[..., 2] = w
    rec[..., 3] = h
    rec[..., 4] = th
    rec[..., 5] = c
    rec[..., 6] = s
    rec[..., 7] = 0.0  # RECTANGLE type id
    rec[..., 8::2] = px
    rec[..., 9::2] = py
    return rec


def inside_rect(px, py, rec, r):
    """Rectangle.inside (env/obstacle.py:62-72). px,py broadcast against rec[..., :]."""
    r = F(r)
    with np.errstate(invalid="ignore"):
        rel_x = px - rec[..., 0]
        rel_y = py - rec[..., 1]
        c, s = rec[..., 5], rec[..., 6]
        rel_xx = np.abs(rel_x * c + rel_y * s) - rec[..., 2] / F(2)
        rel_yy = np.abs(rel_x * s - rel_y * c) - rec[..., 3] / F(2)
        down = (rel_xx < r) & (rel_yy < 0)
        up = (rel_xx < 0) & (rel_yy < r)
        corner = (rel_xx > 0) & (rel_yy > 0)
        circle = np.sqrt(rel_xx * rel_xx + rel_yy * rel_yy) < r
    return down | up | (corner & circle)


def raytrace_alpha(sx, sy, ex, ey, rec):
    """Rectangle.raytracing (env/obstacle.py:74-105): min over 4 edges; NaN-propagating.

    sx..ey: (...,) ray; rec: (..., 16) broadcastable.  Returns alpha (...)."""
    with np.errstate(all="ignore"):
        best = None
        for e in range(4):
            x3, y3 = rec[..., 8 + 2 * e], rec[..., 9 + 2 * e]
            e4 = (e - 1) % 4  # points[[-1, 0, 1, 2]]
            x4, y4 = rec[..., 8 + 2 * e4], rec[..., 9 + 2 * e4]
            det = (sx - ex) * (y4 - y3) - (sy - ey) * (x4 - x3)
            det = np.sign(det) * np.clip(np.abs(det), F(1e-7), F(1e7))
            alpha = ((y4 - y3) * (sx - x3) - (x4 - x3) * (sy - y3)) / det
            beta = (-(sy - ey) * (sx - x3) + (sx - ex) * (sy - y3)) / det
            valid = (alpha <= 1) & (alpha >= 0) & (beta <= 1) & (beta >= 0)
            alpha = valid.astype(F) * alpha + (F(1) - valid.astype(F)) * F(1e6)
            best = alpha if best is None else np.minimum(best, alpha)
    return best.astype(F)


def lidar(pos, obst, ray_tab, top_k):
    """get_lidar + raytracing (env/utils.py:49-79, 115-136) for every agent.

    pos (B, n, 2); obst (B, O, 16); ray_tab (R, 2).  Returns hits (B, n, k, 2)."""
    B, n, _ = pos.shape
    sx = pos[:, :, None, 0]  # (B, n, 1)
    sy = pos[:, :, None, 1]
    ex = (sx + ray_tab[None, None, :, 0]).astype(F)  # (B, n, R)
    ey = (sy + ray_tab[None, None, :, 1]).astype(F)
    O = obst.shape[1]
    if O == 0:
        alpha = np.full(ex.shape, F(1e6), F)
    else:
        rec = obst[:, None, None, :, :]  # (B, 1, 1, O, 16)
        a = raytrace_alpha(sx[..., None], sy[..., None], ex[..., None], ey[..., None], rec)  # (B,n,R,O)
        alpha = np.min(a, axis=-1)  # NaN-propagating
        is_in = inside_rect(pos[:, :, None, 0], pos[:, :, None, 1], obst[:, None, :, :], 0.0).any(axis=-1)
        alpha = (alpha * (F(1) - is_in.astype(F))[..., None]).astype(F)
    order = np.argsort(alpha, axis=-1, kind="stable")[..., :top_k]  # NaN last, stable
    dx = ex - sx
    dy = ey - sy
    hx = sx + dx * alpha
    hy = sy + dy * alpha
    hits = np.stack([np.take_along_axis(hx, order, -1), np.take_along_axis(hy, order, -1)], -1)
    return hits.astype(F), alpha


# ---- dynamics --------------------------------------------------------------------------------
def step_double_integrator(spec, agent, action):
    """agent_step_euler (lidar_env/base.py:142-149, mpe/base.py:129-135)."""
    dt = F(spec.dt)
    xdot = np.concatenate([agent[..., 2:], action * F(10.0)], axis=-1)
    new = xdot * dt + agent
    lo, hi = spec.state_lim()
    return clip(new, lo, hi)


def step_bicycle(spec, agent, action):
    """LidarBicycleTarget.agent_step_euler (lidar_bicycle_target.py:92-111)."""
    dt = F(spec.dt)
    x = agent
    theta = math32.atan2(x[..., 3], x[..., 2])
    theta_next = theta + ((x[..., 4] * action[..., 0]) * dt) * F(10)
    st, ct = math32.sincos(theta)
    sn, cn = math32.sincos(theta_next)
    new = np.stack([
        x[..., 0] + (x[..., 4] * ct) * dt,
        x[..., 1] + (x[..., 4] * st) * dt,
        cn,
        sn,
        x[..., 4] + (action[..., 1] * dt) * F(10.0),
    ], axis=-1).astype(F)
    lo, hi = spec.state_lim()
    return clip(new, lo, hi)


def step_omni(spec, agent, action):
    """LidarOmniTarget.agent_step_euler (lidar_omni_target.py:146-197): omni-wheel agent
    [x, y, cos th, sin th, vx, vy, omega], action [ax, ay, alpha] -> acc = 10 a, alpha = 5 a."""
    dt = F(spec.dt)
    x = agent
    acc_x, acc_y = action[..., 0] * F(10.0), action[..., 1] * F(10.0)
    alpha = action[..., 2] * F(5.0)
    theta = math32.atan2(x[..., 3], x[..., 2])
    new_theta = theta + x[..., 6] * dt
    sn, cn = math32.sincos(new_theta)
    new = np.stack([
        x[..., 0] + x[..., 4] * dt,
        x[..., 1] + x[..., 5] * dt,
        cn,
        sn,
        x[..., 4] + acc_x * dt,
        x[..., 5] + acc_y * dt,
        x[..., 6] + alpha * dt,
    ], axis=-1).astype(F)
    lo, hi = spec.state_lim()
    return clip(new, lo, hi)


def omni_cos_fov(spec):
    """jnp.cos(jnp.deg2rad(fov_angle_deg)) in float32 (lidar_omni_target.py:93-94); cos by the
    shared deterministic fp32 routine (math32), as every other trig term here."""
    beta = F(F(spec.params["fov_angle_deg"]) * F(np.pi / 180))
    return F(math32.sincos(np.array([beta], F))[1][0])


def state2feat(spec, s):
    """LidarBicycleTarget.state2feat (lidar_bicycle_target.py:113-118); identity otherwise."""
    if spec.engine == ENGINE_BICYCLE:
        return np.stack([s[..., 0], s[..., 1], s[..., 4] * s[..., 2], s[..., 4] * s[..., 3]], -1).astype(F)
    return s


# ---- reward / cost ---------------------------------------------------------------------------
def get_reward(spec, agent, goal, action):
    """get_reward: spread (lidar_spread.py:35-52, mpe_spread.py:32-49) or target
    (lidar_target.py:35-52, mpe_target.py:32-49).  Means summed sequentially over agents."""
    n = spec.n
    ap, gp = agent[..., :2], goal[..., :2]
    if spec.goal_mode == GOAL_SPREAD:
        d = norm2d(gp[:, :, None, 0] - ap[:, None, :, 0], gp[:, :, None, 1] - ap[:, None, :, 1]).min(axis=2)
    else:
        d = norm2d(gp[..., 0] - ap[..., 0], gp[..., 1] - ap[..., 1])
    far = (d > F(spec.dist2goal)).astype(F)
    an = norm2d(action[..., 0], action[..., 1])
    an2 = an * an
    s_d = np.zeros(d.shape[0], F)
    s_f = np.zeros(d.shape[0], F)
    s_a = np.zeros(d.shape[0], F)
    for i in range(n):
        s_d = s_d + d[:, i]
        s_f = s_f + far[:, i]
        s_a = s_a + an2[:, i]
    nn = F(n)
    r = F(0) - (s_d / nn) * F(0.01)
    r = r - (s_f / nn) * F(0.001)
    r = r - (s_a / nn) * F(0.0001)
    return r.astype(F)


def _margin(cost, upper):
    eps = F(0.5)
    c = np.where(cost <= 0, cost - eps, cost + eps).astype(F)
    return clip(c, F(-1), F(1)) if upper else np.maximum(c, F(-1)).astype(F)


def agent_min_dist(agent):
    """min_j!=i ||p_i - p_j|| with the eye*1e6 diagonal (lidar_env/base.py:185-187)."""
    n = agent.shape[1]
    ap = agent[..., :2]
    d = norm2d(ap[:, :, None, 0] - ap[:, None, :, 0], ap[:, :, None, 1] - ap[:, None, :, 1])
    d = d + (np.eye(n, dtype=F) * F(1e6))[None]
    return d.min(axis=2)


def get_cost_lidar(spec, agent, hits_cur):
    """LidarEnv.get_cost (lidar_env/base.py:180-207). hits_cur (B, n, k, 2) of the pre-step graph."""
    agent_cost = F(spec.car_r * 2) - agent_min_dist(agent)
    if spec.has_lidar:
        ap = agent[..., :2]
        d = norm2d(hits_cur[..., 0] - ap[:, :, None, 0], hits_cur[..., 1] - ap[:, :, None, 1])
        obs_cost = F(spec.car_r) - d.min(axis=-1)
    else:
        obs_cost = np.zeros_like(agent_cost)
    return _margin(np.stack([agent_cost, obs_cost], -1).astype(F), upper=True)


def get_cost_mpe(spec, agent, obs):
    """MPE.get_cost (mpe/base.py:164-191). obs (B, O, 4) of the pre-step graph."""
    agent_cost = F(spec.car_r * 2) - agent_min_dist(agent)
    if spec.n_obs > 0:
        ap = agent[..., :2]
        d = norm2d(ap[:, :, None, 0] - obs[:, None, :, 0], ap[:, :, None, 1] - obs[:, None, :, 1])
        obs_cost = F(spec.car_r + spec.obs_r) - d.min(axis=2)
    else:
        obs_cost = np.zeros_like(agent_cost)
    return _margin(np.stack([agent_cost, obs_cost], -1).astype(F), upper=False)


def get_reward_omni(spec, agent, goal, action):
    """LidarOmniTarget.get_reward (lidar_omni_target.py:295-336), means summed sequentially."""
    n = spec.n
    d = norm2d(goal[..., 0] - agent[..., 0], goal[..., 1] - agent[..., 1])
    far = (d > F(spec.dist2goal)).astype(F)
    an = norm2d(action[..., 0], action[..., 1])
    terms = [d, far, an * an, action[..., 2] * action[..., 2], agent[..., 6] * agent[..., 6]]
    sums = [np.zeros(d.shape[0], F) for _ in terms]
    for i in range(n):
        for q, t in enumerate(terms):
            sums[q] = sums[q] + t[:, i]
    nn = F(n)
    rp = F(spec.params["rotation_penalty"])
    r = F(0) - (sums[0] / nn) * F(0.01)
    r = r - (sums[1] / nn) * F(0.001)
    r = r - (sums[2] / nn) * F(0.0001)
    r = r - (sums[3] / nn) * rp
    r = r - ((sums[4] / nn) * rp) * F(0.5)  # `.mean() * rotation_penalty * 0.5`, left to right
    return r.astype(F)


def get_cost_omni(spec, agent, hits_all):
    """LidarOmniTarget.get_cost (lidar_omni_target.py:517-649): 5 costs, margin 0.1, clip [-1, 1].

    hits_all (B, n*k, 2): the pre-step graph's hit rows.  Reference quirk kept: the obstacle term
    asks type_states for N - 2n = n*k + 1 rows (the pad node counted), so the extra row is the
    origin and min_dist_obs also covers ||p_i - 0||; and it is the minimum over EVERY agent's hits."""
    n = spec.n
    agent_cost = F(spec.car_r * 2) - agent_min_dist(agent)
    ap = agent[..., :2]
    if spec.has_lidar:
        B = agent.shape[0]
        op = np.concatenate([hits_all, np.zeros((B, 1, 2), F)], axis=1)  # (B, nk+1, 2)
        d = norm2d(op[:, None, :, 0] - ap[:, :, None, 0], op[:, None, :, 1] - ap[:, :, None, 1])
        obs_cost = F(spec.car_r) - d.min(axis=2)
    else:
        obs_cost = np.zeros_like(agent_cost)
    safe = F(-1.0)
    h_a = np.full_like(agent_cost, safe)
    h_r = np.full_like(agent_cost, safe)
    h_c = np.full_like(agent_cost, safe)
    if n > 1:
        pi, pj = agent[:, :-1], agent[:, 1:]
        dx = pj[..., 0] - pi[..., 0]
        dy = pj[..., 1] - pi[..., 1]
        c, s_ = pi[..., 2], pi[..., 3]
        lx = c * dx + s_ * dy  # R_i^T (p_j - p_i), row 0
        ly = (-s_) * dx + c * dy
        nrm = norm2d(lx, ly)
        h_a[:, :-1] = omni_cos_fov(spec) * (nrm + F(1e-8)) - lx
        h_r[:, :-1] = nrm - F(spec.params["max_sensor_range"])
        h_c[:, :-1] = F(spec.params["min_safe_distance"]) - nrm
    cost = np.stack([agent_cost, obs_cost, h_a, h_r, h_c], -1).astype(F)
    eps = F(0.1)
    cost = np.where(cost <= 0, cost - eps, cost + eps).astype(F)
    return clip(cost, F(-1), F(1))


# ---- graph build -----------------------------------------------------------------------------
def build_graph(spec, agent, goal, third):
    """get_graph + edge_blocks + GetGraph.to_padded.

    Lidar: lidar_env/base.py:227-271, lidar_spread.py:54-96 / lidar_target.py:54-96; third = hits (B,n,k,2).
    MPE: mpe/base.py:211-241, mpe_spread.py:51-81 / mpe_target.py:51-80; third = obstacles (B,O,4).
    Padding: utils/graph.py:212-247.  Returns dict(nodes, edges, states, receivers, senders)."""
    B = agent.shape[0]
    n, sd, nd = spec.n, spec.sd, spec.nd
    N, E = spec.n_nodes, spec.n_edges
    t0 = n + spec.ng  # first row after the goal node rows
    pad = N - 1
    nodes = np.zeros((B, N, nd), F)
    states = np.zeros((B, N, sd), F)
    nodes[:, :n, :sd] = agent
    nodes[:, n:t0, :sd] = goal
    states[:, :n] = agent
    states[:, n:t0] = goal
    if spec.engine == ENGINE_MPE:
        O = spec.n_obs
        nodes[:, :n, 6] = 1
        nodes[:, n:t0, 5] = 1
        if O > 0:
            nodes[:, t0:t0 + O, :sd] = third
            nodes[:, t0:t0 + O, 4] = 1
            states[:, t0:t0 + O] = third
    else:
        nodes[:, :n, sd + 2] = 1
        nodes[:, n:t0, sd + 1] = 1
        if spec.has_lidar:
            hits = third.reshape(B, n * spec.top_k, 2)
            nodes[:, t0:t0 + spec.n_hits, :2] = hits
            nodes[:, t0:t0 + spec.n_hits, sd] = 1
            states[:, t0:t0 + spec.n_hits, :2] = hits
    states[:, pad] = -1

    fa = state2feat(spec, agent)
    fg = state2feat(spec, goal)
    ap = agent[..., :2]
    edges, recvs, sends = [], [], []

    def block(feats, mask, ids_recv, ids_send):
        nr, ns = len(ids_recv), len(ids_send)
        r = np.broadcast_to(np.asarray(ids_recv, np.int32)[:, None], (nr, ns))
        s = np.broadcast_to(np.asarray(ids_send, np.int32)[None, :], (nr, ns))
        edges.append(feats.reshape(B, nr * ns, spec.ed))
        recvs.append(np.where(mask, r[None], pad).reshape(B, nr * ns).astype(np.int32))
        sends.append(np.where(mask, s[None], pad).reshape(B, nr * ns).astype(np.int32))

    ids_a = np.arange(n)
    omni = spec.engine == ENGINE_OMNI
    # agent-agent
    feats = fa[:, :, None, :] - fa[:, None, :, :]
    pdx = ap[:, :, None, 0] - ap[:, None, :, 0]
    pdy = ap[:, :, None, 1] - ap[:, None, :, 1]
    if omni:  # lidar_omni_target.py:352-419: [s_i - s_j (7) | critical i -> i+1 | ||p_j^i|| | i_x_j]
        gx, gy = -pdx, -pdy  # p_j - p_i
        c, s_ = agent[:, :, None, 2], agent[:, :, None, 3]
        lx = c * gx + s_ * gy  # R_i^T (p_j - p_i)
        ly = (-s_) * gx + c * gy
        crit = np.zeros((n, n), F)
        if n > 1:
            crit[np.arange(n - 1), np.arange(1, n)] = 1
        feats = np.concatenate([feats[..., :7], np.broadcast_to(crit[None, :, :, None], (B, n, n, 1)),
                                norm2d(lx, ly)[..., None], lx[..., None]], -1).astype(F)
    dist = norm2d(pdx, pdy)
    dist = dist + (np.eye(n, dtype=F) * F(spec.comm_r + 1))[None]
    block(feats, dist < F(spec.comm_r), ids_a, ids_a)
    # agent-goal
    if spec.goal_mode == GOAL_SPREAD:  # every agent to every goal node (landmarks for line / formation)
        block(fa[:, :, None, :] - fg[:, None, :, :], np.ones((B, n, spec.ng), bool), ids_a, n + np.arange(spec.ng))
    else:
        for i in range(n):
            gf = fa[:, i] - fg[:, i]
            if omni:  # first 7 features, zero-padded to edge_dim (lidar_omni_target.py:424-443)
                gf = np.concatenate([gf[:, :7], np.zeros((B, 3), F)], -1)
            block(gf[:, None, None, :], np.ones((B, 1, 1), bool), [i], [n + i])
    # agent-obstacle / agent-lidar
    if spec.engine == ENGINE_MPE:
        O = spec.n_obs
        if O > 0:
            op = third[..., :2]
            d = norm2d(ap[:, :, None, 0] - op[:, None, :, 0], ap[:, :, None, 1] - op[:, None, :, 1])
            # corridor / connect connect every obstacle: jnp.less(dist, comm_radius * 100)
            r_obs = spec.comm_r * 100 if spec.variant in (VARIANT_CORRIDOR, VARIANT_CONNECT) else spec.comm_r
            block(agent[:, :, None, :] - third[:, None, :, :], d < F(r_obs), ids_a, t0 + np.arange(O))
    elif spec.has_lidar:
        k = spec.top_k
        for i in range(n):
            lf = ap[:, i, None, :] - third[:, i]  # (B, k, 2)
            ld = norm2d(lf[..., 0], lf[..., 1])
            # LidarOmniTarget masks hits at comm_radius (lidar_omni_target.py:480), the others at
            # comm_radius - 0.1 (lidar_spread.py:95)
            active = ld < F(spec.comm_r if omni else spec.comm_r - 1e-1)
            feats = np.concatenate([lf, np.zeros((B, k, spec.ed - 2), F)], -1)
            block(feats[:, None], active[:, None], [i], t0 + i * k + np.arange(k))
    out = dict(
        nodes=nodes,
        edges=np.concatenate(edges, 1).astype(F),
        states=states,
        receivers=np.concatenate(recvs, 1),
        senders=np.concatenate(sends, 1),
    )
    assert out["edges"].shape == (B, E, spec.ed), (out["edges"].shape, E)
    return out


def node_type(spec):
    n, N = spec.n, spec.n_nodes
    t = -np.ones(N, np.int32)
    t[:n] = 0
    t[n:n + spec.ng] = 1
    t[n + spec.ng:N - 1] = 2
    return t


# ---- step ------------------------------------------------------------------------------------
def env_step(spec, states, obst, action):
    """LidarEnv.step (lidar_env/base.py:151-174) / MPE.step (mpe/base.py:137-158), batched.

    states: (B, N, sd) states of the current (pre-step) graph; obst: (B, O, 16) rectangles (Lidar)
    or None (MPE reads obstacles from graph states); action (B, n, action_dim).
    Returns dict(graph fields of the next graph, reward (B,), cost (B, n, n_cost), next_agent)."""
    n = spec.n
    t0 = n + spec.ng
    states = np.asarray(states, F)
    agent = states[:, :n]
    goal = states[:, n:t0]
    if spec.variant != VARIANT_NONE:
        from .env_variants import variant_step

        return variant_step(spec, states, obst, action)
    if spec.engine == ENGINE_OMNI:  # action_lim: [-1, -1, -1000] .. [1, 1, 1000] (lidar_omni_target.py:511-521)
        a = clip(np.asarray(action, F), np.array([-1, -1, -1000], F), np.array([1, 1, 1000], F))
        nxt = step_omni(spec, agent, a)
        reward = get_reward_omni(spec, agent, goal, a)
    else:
        a = clip(np.asarray(action, F), F(-1), F(1))
        if spec.engine == ENGINE_BICYCLE:
            nxt = step_bicycle(spec, agent, a)
        else:
            nxt = step_double_integrator(spec, agent, a)
        reward = get_reward(spec, agent, goal, a)
    if spec.engine == ENGINE_MPE:
        obs = states[:, 2 * n:2 * n + spec.n_obs]
        cost = get_cost_mpe(spec, agent, obs)
        g = build_graph(spec, nxt, goal, obs)
    else:
        hits_cur = states[:, 2 * n:2 * n + spec.n_hits, :2].reshape(-1, n, spec.top_k, 2) if spec.has_lidar else None
        if spec.engine == ENGINE_OMNI:
            cost = get_cost_omni(spec, agent, states[:, 2 * n:2 * n + spec.n_hits, :2] if spec.has_lidar else None)
        else:
            cost = get_cost_lidar(spec, agent, hits_cur)
        if spec.has_lidar:
            hits, _ = lidar(nxt[..., :2], obst, ray_table(spec.n_rays, spec.comm_r), spec.top_k)
        else:
            hits = None
        g = build_graph(spec, nxt, goal, hits)
    g.update(reward=reward, cost=cost, next_agent=nxt)
    return g


# ---- reset (sequential per env; reference env/utils.py:139-244) -----------------------------
MAX_ITER = 1024
MPE_OBS_MAX_ITER = 1 << 16  # the reference's MPE obstacle loop is unbounded (mpe/base.py:110-118)


class _EnvRng:
    def __init__(self, seed, env_index):
        self.seed = int(seed)
        self.env = int(env_index)
        self.count = 0

    def uniform(self, lo, hi):
        bits = math32.philox4x32(self.count, self.env, 0, 0, self.seed & 0xFFFFFFFF, (self.seed >> 32) & 0xFFFFFFFF)[0]
        self.count += 1
        return F(math32.uniform(bits, lo, hi))


def _inside_any(px, py, obst, r):
    if obst is None or len(obst) == 0:
        return False
    return bool(inside_rect(F(px), F(py), obst, r).any())


def node_goal_rng(rng, side, n, min_dist, obst):
    """get_node_goal_rng (env/utils.py:139-244) for one env, dim=2, max_travel=None.

    Keeps the reference quirks: candidates are compared against ALL n rows including the
    zero-initialised unplaced ones (utils.py:151-152, 171); a failure restarts from agent 0."""
    r_in = F(min_dist / 2)  # Python float min_dist/2, cast once (utils.py:173, 195)
    min_dist = F(min_dist)
    states = np.zeros((n, 2), F)
    goals = np.zeros((n, 2), F)
    agent_id = 0
    while agent_id < n:
        cand = np.array([rng.uniform(0, side), rng.uniform(0, side)], F)
        it = 0
        while True:
            dmin = norm2d(states[:, 0] - cand[0], states[:, 1] - cand[1]).min()
            collide = dmin <= min_dist
            inside = _inside_any(cand[0], cand[1], obst, r_in)
            if not (collide or inside) or it >= MAX_ITER:
                break
            it += 1
            cand = np.array([rng.uniform(0, side), rng.uniform(0, side)], F)
        n_iter_agent = it
        states[agent_id] = cand
        g = np.array([rng.uniform(0, side), rng.uniform(0, side)], F)
        it = 0
        while True:
            dmin = norm2d(goals[:, 0] - g[0], goals[:, 1] - g[1]).min()
            collide = dmin <= min_dist
            inside = _inside_any(g[0], g[1], obst, r_in)
            outside = bool((g < 0).any() or (g > F(side)).any())
            if not (collide or inside or outside) or it >= MAX_ITER:
                break
            it += 1
            g = np.array([rng.uniform(0, side), rng.uniform(0, side)], F)
        goals[agent_id] = g
        agent_id += 1
        if n_iter_agent >= MAX_ITER or it >= MAX_ITER:
            agent_id = 0
            states[:] = 0
            goals[:] = 0
    return states, goals


def min_dist_for(spec):
    if spec.engine == ENGINE_OMNI:  # jnp.maximum(2.2 r, D) (lidar_omni_target.py:237-240), float32
        return float(max(F(2.2 * spec.car_r), F(spec.params["min_safe_distance"])))
    return 2.2 * spec.car_r if spec.engine != ENGINE_MPE else 2 * spec.car_r


def env_reset(spec, seed, n_env, env_offset=0):
    """reset (lidar_env/base.py:89-124; lidar_bicycle_target.py:60-90; mpe/base.py:81-127).

    Returns (agent (B,n,sd), goal (B,n,sd), obst (B,O,16) or MPE obstacle states (B,O,4)); the variants
    (oracle/env_variants.py) return their goal-node rows (B, ng, sd) as `goal`."""
    if spec.variant != VARIANT_NONE:
        from .env_variants import variant_reset

        return variant_reset(spec, seed, n_env, env_offset)
    n, sd, O = spec.n, spec.sd, spec.n_obs
    area = spec.area
    md = min_dist_for(spec)
    agents = np.zeros((n_env, n, sd), F)
    goals = np.zeros((n_env, n, sd), F)
    third = np.zeros((n_env, O, OBST_FIELDS if spec.engine != ENGINE_MPE else 4), F)
    for b in range(n_env):
        rng = _EnvRng(seed, env_offset + b)
        if spec.engine == ENGINE_MPE:
            st, gl = node_goal_rng(rng, area, n, md, None)
            agents[b, :, :2] = st
            goals[b, :, :2] = gl
            lo3, hi3 = 3 * spec.car_r, area - 3 * spec.car_r
            for o in range(O):
                cand = np.array([rng.uniform(0, area), rng.uniform(0, area)], F)
                it = 0
                while it < MPE_OBS_MAX_ITER:
                    da = norm2d(st[:, 0] - cand[0], st[:, 1] - cand[1]).min()
                    dg = norm2d(gl[:, 0] - cand[0], gl[:, 1] - cand[1]).min()
                    bad = (da <= F(spec.car_r + spec.obs_r)) or (dg <= F(spec.car_r * 2 + spec.obs_r)) or \
                        bool((cand < F(lo3)).any() or (cand > F(hi3)).any())
                    if not bad:
                        break
                    cand = np.array([rng.uniform(lo3, hi3), rng.uniform(lo3, hi3)], F)
                    it += 1
                third[b, o, :2] = cand
            continue
        obst = None
        if O > 0:
            c = np.array([[rng.uniform(0, area), rng.uniform(0, area)] for _ in range(O)], F)
            lens = np.array([[rng.uniform(*spec.obs_len_range), rng.uniform(*spec.obs_len_range)] for _ in range(O)], F)
            if spec.engine == ENGINE_BICYCLE:
                th = np.array([rng.uniform(-np.pi, np.pi) for _ in range(O)], F)
            else:
                th = np.array([rng.uniform(0, 2 * np.pi) for _ in range(O)], F)
            obst = make_rectangles(c, lens[:, 0], lens[:, 1], th)
            third[b] = obst
        st, gl = node_goal_rng(rng, area, n, md, obst)
        agents[b, :, :2] = st
        goals[b, :, :2] = gl
        if spec.engine == ENGINE_BICYCLE:
            hd = np.array([rng.uniform(0, 2 * np.pi) for _ in range(n)], F)
            s, c = math32.sincos(hd)
            agents[b, :, 2] = c
            agents[b, :, 3] = s
        if spec.engine == ENGINE_OMNI:  # chain headings (lidar_omni_target.py:246-272)
            for i in range(n - 1):
                dx, dy = F(st[i + 1, 0] - st[i, 0]), F(st[i + 1, 1] - st[i, 1])
                nrm = F(norm2d(np.array([dx], F), np.array([dy], F))[0] + F(1e-8))
                agents[b, i, 2] = F(dx / nrm)
                agents[b, i, 3] = F(dy / nrm)
            th = np.array([rng.uniform(0, 2 * np.pi)], F)  # last agent (or the only one): random heading
            s, c = math32.sincos(th)
            agents[b, n - 1, 2] = c[0]
            agents[b, n - 1, 3] = s[0]
    return agents, goals, third


def initial_graph(spec, agents, goals, third):
    """The graph `reset` returns: get_lidar_data + get_graph on the sampled state."""
    if spec.engine == ENGINE_MPE:
        return build_graph(spec, agents, goals, third)
    hits = None
    if spec.has_lidar:
        hits, _ = lidar(agents[..., :2], third, ray_table(spec.n_rays, spec.comm_r), spec.top_k)
    return build_graph(spec, agents, goals, hits)

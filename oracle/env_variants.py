"""NumPy restatement of the reference's environment VARIANTS (hot path 1).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  float32, one rounding per operation in the
reference's order, like oracle/env.py, whose geometry / graph helpers this module reuses:

  LidarLine        dgppo/env/lidar_env/lidar_line.py      2 landmark goal nodes, n reward goals on
                                                          the segment, rejection-placed obstacles
  MPELine          dgppo/env/mpe/mpe_line.py              same goal rule (n <= 3: interior points)
  MPEFormation     dgppo/env/mpe/mpe_formation.py         1 landmark, reward goals on a circle
  MPECorridor      dgppo/env/mpe/mpe_corridor.py          2 fixed wall obstacles, goals across them
  MPEConnectSpread dgppo/env/mpe/mpe_connect_spread.py    connectivity cost (n_cost 3), 1 obstacle

RNG: the reference's jax.random keys are replaced by the per-env Philox stream of oracle/env.py
(_EnvRng); the draw ORDER below is this port's definition (the HIP reset kernel draws in the same
order).  Unbounded reference rejection loops are capped at 65536 candidates."""
from __future__ import annotations

import numpy as np

from . import math32
from .env import (F, ENGINE_MPE, VARIANT_CONNECT, VARIANT_CORRIDOR, VARIANT_FORMATION, VARIANT_LINE, MAX_ITER,
                  _EnvRng, agent_min_dist, build_graph, clip, inside_rect, lidar, make_rectangles, norm2d, ray_table,
                  step_double_integrator)

LOOP_CAP = 1 << 16


def linspace32(start, stop, num):
    """jnp.linspace(start, stop, num) in float32: start * (1 - s) + stop * s, s = i / (num - 1),
    the endpoint set to stop (the form of oracle/env.py ray_thetas)."""
    start, stop = F(start), F(stop)
    if num == 1:
        return np.array([start], F)
    div = num - 1
    s = (np.arange(div, dtype=F) / F(div)).astype(F)
    return np.concatenate([start * (F(1) - s) + stop * s, [stop]]).astype(F)


def goals_inner(spec):
    """mpe_line.py:112-121: for n <= 3 the goals are the n interior points of the segment."""
    return spec.engine == ENGINE_MPE and spec.n <= 3


def landmark2goal(spec, landmarks):
    """(B, ng, >=2) goal-node rows -> (B, n, 2) reward goals.
    line: l0 + arange(...)[:, None] * (l1 - l0) / n_interval (lidar_line.py:137-142, mpe_line.py:112-121),
    formation: l + R [cos th, sin th], th = linspace(0, 2 pi, n + 1)[:-1] (mpe_formation.py:92-96)."""
    n = spec.n
    lm = np.asarray(landmarks, F)[..., :2]
    if spec.variant == VARIANT_LINE:
        d = (lm[:, 1] - lm[:, 0]).astype(F)  # (B, 2)
        if goals_inner(spec):
            k = np.arange(1, n + 1, dtype=F)
            m = F(n + 1)
        else:
            k = np.arange(0, n, dtype=F)
            m = F(n - 1)
        return (lm[:, :1] + (k[None, :, None] * d[:, None, :]) / m).astype(F)
    if spec.variant == VARIANT_FORMATION:
        th = linspace32(0.0, 2 * np.pi, n + 1)[:-1]
        s, c = math32.sincos(th)
        off = np.stack([c, s], -1).astype(F)  # (n, 2)
        return (lm[:, :1] + F(spec.comm_r) * off[None]).astype(F)
    return lm


def reward_spread(spec, agent, goals, action):
    """MPESpread/LidarSpread.get_reward with the given reward goals (B, n, 2): each goal's nearest
    agent, means summed sequentially over the n goals / agents."""
    n = spec.n
    ap = agent[..., :2]
    d = norm2d(goals[:, :, None, 0] - ap[:, None, :, 0], goals[:, :, None, 1] - ap[:, None, :, 1]).min(axis=2)
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


def cost_variant(spec, agent, third):
    """get_cost: LidarLine = LidarEnv (lidar_env/base.py:180-207, third = current hits (B, n, k, 2));
    MPE variants = MPE.get_cost (mpe/base.py:164-191); MPEConnectSpread adds the connectivity cost
    max_i(min_j ||p_i - p_j|| - connect_radius) and clips to [-1, 1] (mpe_connect_spread.py:104-138)."""
    md = agent_min_dist(agent)
    agent_cost = F(spec.car_r * 2) - md
    ap = agent[..., :2]
    if spec.engine != ENGINE_MPE:
        if spec.has_lidar:
            d = norm2d(third[..., 0] - ap[:, :, None, 0], third[..., 1] - ap[:, :, None, 1])
            obs_cost = F(spec.car_r) - d.min(axis=-1)
        else:
            obs_cost = np.zeros_like(agent_cost)
        comps = [agent_cost, obs_cost]
        upper = True
    else:
        if spec.n_obs > 0:
            d = norm2d(ap[:, :, None, 0] - third[:, None, :, 0], ap[:, :, None, 1] - third[:, None, :, 1])
            obs_cost = F(spec.car_r + spec.obs_r) - d.min(axis=2)
        else:
            obs_cost = np.zeros_like(agent_cost)
        comps = [agent_cost, obs_cost]
        upper = False
        if spec.variant == VARIANT_CONNECT:
            con = (md - F(spec.params["connect_radius"])).astype(F)
            cmax = con[:, 0]
            for i in range(1, spec.n):  # .max(), NaN-propagating
                cmax = np.where(np.isnan(cmax) | (cmax >= con[:, i]), cmax, con[:, i]).astype(F)
            comps.append(np.repeat(cmax[:, None], spec.n, 1))
            upper = True
    cost = np.stack(comps, -1).astype(F)
    eps = F(0.5)
    cost = np.where(cost <= 0, cost - eps, cost + eps).astype(F)
    return clip(cost, F(-1), F(1)) if upper else np.maximum(cost, F(-1)).astype(F)


def variant_step(spec, states, obst, action):
    """The variants' step (LidarEnv.step / MPE.step with the variant's reward / cost / graph)."""
    n, t0 = spec.n, spec.n + spec.ng
    states = np.asarray(states, F)
    agent = states[:, :n]
    grow = states[:, n:t0]
    a = clip(np.asarray(action, F), F(-1), F(1))
    nxt = step_double_integrator(spec, agent, a)
    reward = reward_spread(spec, agent, landmark2goal(spec, grow), a)
    if spec.engine == ENGINE_MPE:
        obs = states[:, t0:t0 + spec.n_obs]
        cost = cost_variant(spec, agent, obs)
        g = build_graph(spec, nxt, grow, obs)
    else:
        hits_cur = states[:, t0:t0 + spec.n_hits, :2].reshape(-1, n, spec.top_k, 2) if spec.has_lidar else None
        cost = cost_variant(spec, agent, hits_cur)
        hits = lidar(nxt[..., :2], obst, ray_table(spec.n_rays, spec.comm_r), spec.top_k)[0] if spec.has_lidar else None
        g = build_graph(spec, nxt, grow, hits)
    g.update(reward=reward, cost=cost, next_agent=nxt)
    return g


# ---- resets ------------------------------------------------------------------------------------
def node_goal_rng_y(rng, side, side_y, n, min_dist):
    """get_node_goal_rng (env/utils.py:139-244) with side_length_y and no obstacles: candidates
    (uniform(0, side), uniform(0, side_y)); the goal bound check stays `goal > side_length`."""
    min_dist = F(min_dist)
    states = np.zeros((n, 2), F)
    goals = np.zeros((n, 2), F)
    agent_id = 0

    def draw():
        return np.array([rng.uniform(0, side), rng.uniform(0, side_y)], F)

    while agent_id < n:
        cand = draw()
        it = 0
        while True:
            dmin = norm2d(states[:, 0] - cand[0], states[:, 1] - cand[1]).min()
            if not (dmin <= min_dist) or it >= MAX_ITER:
                break
            it += 1
            cand = draw()
        n_iter_agent = it
        states[agent_id] = cand
        g = draw()
        it = 0
        while True:
            dmin = norm2d(goals[:, 0] - g[0], goals[:, 1] - g[1]).min()
            outside = bool((g < 0).any() or (g > F(side)).any())
            if not (dmin <= min_dist or outside) or it >= MAX_ITER:
                break
            it += 1
            g = draw()
        goals[agent_id] = g
        agent_id += 1
        if n_iter_agent >= MAX_ITER or it >= MAX_ITER:
            agent_id = 0
            states[:] = 0
            goals[:] = 0
    return states, goals


def line_min_dist(spec):
    r = spec.car_r
    if spec.engine == ENGINE_MPE and spec.n <= 3:
        return spec.n * 5 * r  # mpe_line.py:48-49
    return (spec.n - 2) * 6 * r  # lidar_line.py:54, mpe_line.py:51


def landmarks_line(spec, rng):
    """Two landmarks (lidar_line.py:53-84, mpe_line.py:47-83): l0 on a rotated edge strip, l1 at
    distance >= min_dist.  Draws: l0 (2) [+ region (1)], then l1 candidates (2 each)."""
    area = spec.area
    md = line_min_dist(spec)
    if spec.engine == ENGINE_MPE and spec.n <= 3:
        l0 = np.array([rng.uniform(0, area), rng.uniform(0, area)], F)
    else:
        side = area - md
        if side < 0:
            raise ValueError("The area size is too small to place the landmarks.")
        u = np.array([rng.uniform(0, area - side), rng.uniform(0, side)], F)
        c = (u - np.array([area / 2, 0], F)).astype(F)
        c = (c + np.array([0, area / 2 - side], F)).astype(F)
        region = min(int(rng.uniform(0, 4)), 3)  # jr.randint(0, 4)
        ang = F(F(region) * F(np.pi)) / F(2)
        s, co = math32.sincos(np.array([ang], F))
        s, co = F(s[0]), F(co[0])
        rx = F(F(co * c[0]) + F(F(-s) * c[1]))
        ry = F(F(s * c[0]) + F(co * c[1]))
        l0 = np.array([F(rx + F(area / 2)), F(ry + F(area / 2))], F)
    l1 = np.array([rng.uniform(0, area), rng.uniform(0, area)], F)
    it = 0
    while norm2d(l1[0:1] - l0[0], l1[1:2] - l0[1])[0] < F(md) and it < LOOP_CAP:
        l1 = np.array([rng.uniform(0, area), rng.uniform(0, area)], F)
        it += 1
    return np.stack([l0, l1]).astype(F)


def mpe_obstacles(spec, rng, states, goals):
    """MPE obstacle rejection (mpe/base.py:92-118, the line / formation copies): candidate uniform(0, area)
    first, then uniform(3r, area - 3r); invalid when within r + obs_r of an agent, 2r + obs_r of a goal,
    or outside [3r, area - 3r]."""
    area, r, orr = spec.area, spec.car_r, spec.obs_r
    lo3, hi3 = 3 * r, area - 3 * r
    out = np.zeros((spec.n_obs, 4), F)
    for o in range(spec.n_obs):
        cand = np.array([rng.uniform(0, area), rng.uniform(0, area)], F)
        it = 0
        while it < LOOP_CAP:
            da = norm2d(states[:, 0] - cand[0], states[:, 1] - cand[1]).min()
            dg = norm2d(goals[:, 0] - cand[0], goals[:, 1] - cand[1]).min()
            bad = (da <= F(r + orr)) or (dg <= F(r * 2 + orr)) or bool((cand < F(lo3)).any() or (cand > F(hi3)).any())
            if not bad:
                break
            cand = np.array([rng.uniform(lo3, hi3), rng.uniform(lo3, hi3)], F)
            it += 1
        out[o, :2] = cand
    return out


def lidar_line_obstacles(spec, rng, points):
    """lidar_line.py:86-122: per obstacle pos (2), side lengths (2), theta in [0, pi) (1), redrawn
    until no agent / goal point is inside it inflated by 1.1 car radii."""
    area = spec.area
    lo, hi = spec.obs_len_range
    recs = np.zeros((spec.n_obs, 16), F)
    r_in = F(spec.car_r * 1.1)
    for o in range(spec.n_obs):
        it = 0
        while True:
            c = np.array([rng.uniform(0, area), rng.uniform(0, area)], F)
            wl = np.array([rng.uniform(lo, hi), rng.uniform(lo, hi)], F)
            th = np.array([rng.uniform(0, np.pi)], F)
            rec = make_rectangles(c[None], wl[:1], wl[1:], th)
            inside = bool(inside_rect(points[:, 0], points[:, 1], rec, r_in).any())
            if not inside or it >= LOOP_CAP:
                break
            it += 1
        recs[o] = rec[0]
    return recs


def variant_reset(spec, seed, n_env, env_offset=0):
    """reset of the variants.  Returns (agent (B, n, 4), goal rows (B, ng, 4), third) with third the
    Lidar obstacle records (B, O, 16) or the MPE obstacle states (B, O, 4)."""
    n, ng, O, area, r = spec.n, spec.ng, spec.n_obs, spec.area, spec.car_r
    agents = np.zeros((n_env, n, 4), F)
    grows = np.zeros((n_env, ng, 4), F)
    third = np.zeros((n_env, O, 16 if spec.engine != ENGINE_MPE else 4), F)
    for b in range(n_env):
        rng = _EnvRng(seed, env_offset + b)
        if spec.variant in (VARIANT_LINE, VARIANT_FORMATION):
            st, _ = node_goal_rng_y(rng, area, area, n, 2 * r)
            if spec.variant == VARIANT_LINE:
                lm = landmarks_line(spec, rng)
            else:  # mpe_formation.py:47-52
                R = spec.comm_r
                lm = np.array([[rng.uniform(R + 2 * r, area - R - 2 * r), rng.uniform(R + 2 * r, area - R - 2 * r)]], F)
            goals = landmark2goal(spec, lm[None])[0]
            if spec.engine == ENGINE_MPE:
                third[b] = mpe_obstacles(spec, rng, st, goals)
            elif O > 0:
                third[b] = lidar_line_obstacles(spec, rng, np.concatenate([st, goals]).astype(F))
            agents[b, :, :2] = st
            grows[b, :, :2] = lm
            continue
        orr = spec.obs_r
        side_y = (area - orr * 2) / 2 - 1.5 * r
        shift = np.array([0.0, area - (area - orr * 2) / 2 + 1.5 * r], F)
        if spec.variant == VARIANT_CORRIDOR:  # mpe_corridor.py:40-53
            st, gl = node_goal_rng_y(rng, area, side_y, n, 2 * r)
            gl = (gl + shift).astype(F)
            third[b, :, :2] = np.array([[orr, area / 2], [area - orr, area / 2]], F)
        else:  # VARIANT_CONNECT, mpe_connect_spread.py:47-94
            cr = F(spec.params["connect_radius"])
            it = 0
            while True:
                st, gl = node_goal_rng_y(rng, area, side_y, n, 2.3 * r)
                gl = (gl + shift).astype(F)
                md_a = agent_min_dist(st[None])[0]
                md_g = agent_min_dist(gl[None])[0]
                bad = bool((md_a > cr).any() or (md_a < F(2 * r)).any() or (md_g > cr).any())
                it += 1
                if not bad or it >= LOOP_CAP:
                    break
            third[b, 0, :2] = np.array([rng.uniform(orr, area - orr), area / 2], F)
        agents[b, :, :2] = st
        grows[b, :, :2] = gl
    return agents, grows, third

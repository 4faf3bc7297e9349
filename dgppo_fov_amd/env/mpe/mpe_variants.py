"""The MPE variants (dgppo/env/mpe/): MPELine, MPEFormation, MPECorridor, MPEConnectSpread.  Each is a
SPREAD double-integrator MPE env whose step / reset run in the variant kernels of libdgppo_hip.so; the
Python side only describes the variant in the env cfg (include/dgppo_hip.h, ABI 6)."""
from __future__ import annotations

from typing import Tuple

import torch

from ... import _lib
from .mpe_spread import MPESpread


class MPELine(MPESpread):
    """mpe_line.py: two landmark goal nodes, reward goals on the segment (n <= 3: the n interior points,
    else evenly spaced including both ends, :112-121); landmark / obstacle placement :38-110."""
    PARAMS = dict(MPESpread.PARAMS)

    def __init__(self, num_agents, area_size=None, max_step=128, dt=0.03, params=None, device=None):
        area = type(self).PARAMS["default_area_size"] if area_size is None else area_size
        p = type(self).PARAMS if params is None else params
        if num_agents > 3 and area - (num_agents - 2) * 6 * p["car_radius"] < 0:  # mpe_line.py:55-57
            raise ValueError("The area size is too small to place the landmarks.")
        super().__init__(num_agents, area_size, max_step, dt, params, device)

    def _n_goals(self) -> int:
        return 2

    def _engine_cfg(self, c) -> None:
        n, r, area = self._num_agents, self._params["car_radius"], self._area_size
        c.variant = _lib.DGPPO_VARIANT_LINE
        c.goals_inner = 1 if n <= 3 else 0
        md = n * 5 * r if n <= 3 else (n - 2) * 6 * r
        c.line_min_dist = md
        if n > 3:
            side = area - md
            c.line_box_x, c.line_box_y, c.line_off_y = area - side, side, area / 2 - side


class MPEFormation(MPESpread):
    """mpe_formation.py: one landmark goal node; the reward goals are n points on the circle of radius
    comm_radius around it (landmark2goal :92-96); landmark uniform in [R + 2r, area - R - 2r] (:46-52)."""
    PARAMS = dict(MPESpread.PARAMS)

    def _n_goals(self) -> int:
        return 1

    def _engine_cfg(self, c) -> None:
        R, r, area = self._params["comm_radius"], self._params["car_radius"], self._area_size
        c.variant = _lib.DGPPO_VARIANT_FORMATION
        c.goal_radius = R
        c.formation_lo, c.formation_hi = R + 2 * r, area - R - 2 * r


class _TallMPE(MPESpread):
    """Corridor / connect: agents start below the obstacle row, goals above it (y up to 2 area)."""

    def state_lim(self, state=None):
        a = self.area_size
        return torch.tensor([0.0, 0.0, -1.0, -1.0]), torch.tensor([a, 2 * a, 1.0, 1.0])

    def _tall_cfg(self, c) -> None:
        r, orr, area = self._params["car_radius"], self._params["obs_radius"], self._area_size
        c.obs_edge_radius = self._params["comm_radius"] * 100  # always connected (mpe_corridor.py:90)
        c.sample_side_y = (area - orr * 2) / 2 - 1.5 * r
        c.goal_shift_y = area - (area - orr * 2) / 2 + 1.5 * r
        c.obs_x_hi = area - orr


class MPECorridor(_TallMPE):
    """mpe_corridor.py: two fixed wall obstacles of radius (area - corridor_width) / 4 leave a corridor;
    agents start below, goals above (reset :39-58)."""
    PARAMS = {"car_radius": 0.05, "comm_radius": 0.5, "default_area_size": 1.0, "dist2goal": 0.01, "n_obs": 2,
              "corridor_width": 0.2}

    def __init__(self, num_agents, area_size=None, max_step=128, dt=0.03, params=None, device=None):
        area = type(self).PARAMS["default_area_size"] if area_size is None else area_size
        p = dict(type(self).PARAMS if params is None else params)
        if p["n_obs"] != 2:
            p["n_obs"] = 2
            print("WARNING: n_obs is set to 2 for MPECorridor.")
        p["obs_radius"] = (area - p["corridor_width"]) / 4  # mpe_corridor.py:37
        super().__init__(num_agents, area_size, max_step, dt, p, device)

    def _engine_cfg(self, c) -> None:
        c.variant = _lib.DGPPO_VARIANT_CORRIDOR
        self._tall_cfg(c)


class MPEConnectSpread(_TallMPE):
    """mpe_connect_spread.py: one large obstacle between the start and goal regions and a connectivity
    cost (third cost: max over agents of the nearest-neighbour distance minus connect_radius, :104-138)."""
    PARAMS = {"car_radius": 0.05, "comm_radius": 0.5, "default_area_size": 1.0, "dist2goal": 0.01, "n_obs": 1,
              "obs_radius": 0.25, "connect_radius": 0.45}

    def __init__(self, num_agents, area_size=None, max_step=128, dt=0.03, params=None, device=None):
        p = dict(type(self).PARAMS if params is None else params)
        if p["n_obs"] != 1:
            p["n_obs"] = 1
            print("WARNING: n_obs is set to 1 for MPEConnectSpread.")
        super().__init__(num_agents, area_size, max_step, dt, p, device)

    @property
    def n_cost(self) -> int:
        return 3

    @property
    def cost_components(self) -> Tuple[str, ...]:
        return "agent collisions", "obs collisions", "connectivity"

    def _engine_cfg(self, c) -> None:
        c.variant = _lib.DGPPO_VARIANT_CONNECT
        c.connect_radius = self._params["connect_radius"]
        c.c_connect_min = 2.3 * self._params["car_radius"]
        self._tall_cfg(c)

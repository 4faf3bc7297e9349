"""LidarEnv (dgppo/env/lidar_env/base.py:35-281): double-integrator agents with a 32-ray LiDAR
against rectangular obstacles; the top-k hits become graph nodes.  Step/reset run in
libdgppo_hip.so (one fused kernel each)."""
from __future__ import annotations

from typing import NamedTuple, Optional

import torch

from ... import _lib
from ..base import MultiAgentEnv
from ..obstacle import OBST_FIELDS, Rectangle


class LidarEnvState(NamedTuple):
    agent: torch.Tensor  # (..., n, state_dim)   view of graph.states rows [0, n)
    goal: torch.Tensor  # (..., n, state_dim)    view of graph.states rows [n, 2n)
    obstacle: Optional[Rectangle]  # (..., O, 16) packed records

    @property
    def n_agent(self) -> int:
        return self.agent.shape[-2]


class LidarEnv(MultiAgentEnv):
    ENGINE = _lib.DGPPO_ENGINE_LIDAR
    PARAMS = {
        "car_radius": 0.05,
        "comm_radius": 0.5,
        "n_rays": 32,
        "obs_len_range": [0.1, 0.3],
        "n_obs": 3,
        "default_area_size": 1.5,
        "dist2goal": 0.01,
        "top_k_rays": 8,
    }

    def __init__(self, num_agents: int, area_size: Optional[float] = None, max_step: int = 128,
                 dt: float = 0.03, params: dict = None, device=None):
        area_size = type(self).PARAMS["default_area_size"] if area_size is None else area_size
        super().__init__(num_agents, area_size, max_step, dt, params, device)

    @property
    def state_dim(self) -> int:
        return 4  # x, y, vx, vy

    @property
    def node_dim(self) -> int:
        return 7  # state (4) + indicator: agent 001, goal 010, obstacle 100

    def state_lim(self, state=None):
        return torch.tensor([0.0, 0.0, -0.5, -0.5]), torch.tensor([self.area_size, self.area_size, 0.5, 0.5])

    def _obstacle_fields(self) -> int:
        return OBST_FIELDS if self.n_obs > 0 else 0

    def _env_states(self, states, obstacles):
        n = self.num_agents
        ob = None
        if obstacles is not None:
            extra = states.dim() - 2 - (obstacles.dim() - 2)  # e.g. (B, T) graph views over (B,) obstacles
            if extra > 0:
                obstacles = obstacles.reshape(obstacles.shape[:1] + (1,) * extra + obstacles.shape[1:]).expand(
                    tuple(states.shape[:-2]) + tuple(obstacles.shape[1:]))
            ob = Rectangle(obstacles)
        return LidarEnvState(states[..., :n, :], states[..., n:n + self.num_goals, :], ob)

    def _obstacles_of(self, graph):
        if self.n_obs == 0:
            return None
        ob = graph.env_states.obstacle
        if ob is None:
            raise ValueError("LidarEnv graph carries no obstacles (env_states.obstacle is None)")
        t = ob.packed
        if t.stride(-1) != 1 or t.stride(-2) != OBST_FIELDS:
            raise ValueError("obstacle records must be contiguous per env")
        return t

"""MPE (dgppo/env/mpe/base.py:30-251): double-integrator particles with point obstacles that are
graph nodes.  Step/reset run in libdgppo_hip.so."""
from __future__ import annotations

from typing import NamedTuple, Optional

import torch

from ... import _lib
from ..base import MultiAgentEnv


class MPEEnvState(NamedTuple):
    agent: torch.Tensor  # (..., n, 4) view of graph.states rows [0, n)
    goal: torch.Tensor  # (..., n, 4)  rows [n, 2n)
    obs: torch.Tensor  # (..., O, 4)   rows [2n, 2n + O)

    @property
    def n_agent(self) -> int:
        return self.agent.shape[-2]


class MPE(MultiAgentEnv):
    ENGINE = _lib.DGPPO_ENGINE_MPE
    PARAMS = {
        "car_radius": 0.05,
        "comm_radius": 0.5,
        "n_obs": 3,
        "obs_radius": 0.05,
        "default_area_size": 1.5,
        "dist2goal": 0.01,
    }

    def __init__(self, num_agents: int, area_size: Optional[float] = None, max_step: int = 128,
                 dt: float = 0.03, params: dict = None, device=None):
        area_size = type(self).PARAMS["default_area_size"] if area_size is None else area_size
        super().__init__(num_agents, area_size, max_step, dt, params, device)

    def state_lim(self, state=None):
        return torch.tensor([0.0, 0.0, -1.0, -1.0]), torch.tensor([self.area_size, self.area_size, 1.0, 1.0])

    def _env_states(self, states, obstacles):
        n, ng, O = self.num_agents, self.num_goals, self.n_obs
        return MPEEnvState(states[..., :n, :], states[..., n:n + ng, :], states[..., n + ng:n + ng + O, :])

"""VMAS contact-physics envs (dgppo/env/vmas/): VMASWheel (3 agents push a line rotating about the origin
to a goal angle past an avoid sector) and VMASReverseTransport (3 agents inside a hollow box carry it to a
goal past 3 obstacles).  Reset / step / rollout run the HIP kernels of csrc/vmas.hip through the
same dgppo_env_* C-ABI as every other env (engines DGPPO_ENGINE_VMAS_WHEEL / _TRANSPORT).

Layout differences from the reference (documented in include/dgppo_hip.h):
  * graph.states is (.., 4, 4): the agents' [x, y, vx, vy] rows plus the moving body in the pad row
    (the reference pads a 0-wide state); env_states are views of it and of a per-env record
    (.., 1, 8) holding the per-episode goal / avoid / obstacle constants.
  * jax.random keys are Philox streams (one per jax.random.split key of reset).
"""
from __future__ import annotations

import ctypes
from typing import NamedTuple, Optional, Tuple

import torch

from ... import _lib
from ...utils.graph import GraphsTuple
from ..base import MultiAgentEnv


class VMASWheelState(NamedTuple):  # vmas_wheel.py:25-32 (a_contact_force: node columns 7:9)
    line_angle: torch.Tensor  # (...,)
    line_angvel: torch.Tensor
    a_pos: torch.Tensor  # (..., 3, 2)
    a_vel: torch.Tensor
    a_contact_force: Optional[torch.Tensor]  # (..., 3, 2)
    goal_angle: torch.Tensor
    avoid_angle: torch.Tensor
    record: torch.Tensor  # (..., 1, 8) the packed per-env constants the kernels read


class VMASReverseTransportState(NamedTuple):  # vmas_reverse_transport.py:23-29
    box_pos: torch.Tensor  # (..., 2)
    box_vel: torch.Tensor
    a_pos: torch.Tensor  # (..., 3, 2)
    a_vel: torch.Tensor
    goal_pos: torch.Tensor  # (..., 2)
    o_pos: torch.Tensor  # (..., 3, 2)
    record: torch.Tensor


class VMASEnv(MultiAgentEnv):
    """Shared plumbing of the two VMAS envs (3 agents, 4 nodes, 9 agent-agent edges)."""

    AGENT = 0
    PARAMS = {"comm_radius": 0.4, "default_area_size": 0.8, "dist2goal": 0.01, "agent_radius": 0.03}
    HALF_WIDTH = 1.0
    N_OBS = 0
    NODE_DIM = 13
    # only agent rows and the all-zero pad row exist: the agent-mode layers' raw sender rows need one column
    nonagent_feature_cols = (0,)

    def __init__(self, num_agents: int, area_size: Optional[float] = None, max_step: int = 64, dt: float = 0.1,
                 params: dict = None, device=None):
        assert num_agents == 3, f"{type(self).__name__} only supports 3 agents."
        self.half_width = self.HALF_WIDTH
        self.agent_radius = 0.03
        super().__init__(3, 2 * self.HALF_WIDTH, max_step, dt, params, device)

    def _n_goals(self) -> int:
        return 0

    @property
    def n_obs(self) -> int:
        return self.N_OBS

    @property
    def state_dim(self) -> int:
        return 4  # x, y, vx, vy

    @property
    def node_dim(self) -> int:
        return self.NODE_DIM

    @property
    def edge_dim(self) -> int:
        return 4

    @property
    def action_dim(self) -> int:
        return 2

    @property
    def n_cost(self) -> int:
        return 2

    def state_lim(self, state=None):
        return None  # the reference's state_lim is `pass`

    def _obstacle_fields(self) -> int:
        return _lib.DGPPO_VMAS_FIELDS

    def _obstacle_rows(self) -> int:
        return 1

    def _make_cfg(self) -> _lib.EnvCfg:
        p = self._params
        c = _lib.EnvCfg()
        c.engine = self.ENGINE
        c.goal_mode = _lib.DGPPO_GOAL_SPREAD
        c.n_agents = self._num_agents
        c.dt = self._dt
        c.comm_radius = p["comm_radius"]
        c.car_radius = p["agent_radius"]
        c.area_size = self._area_size
        c.dist2goal = p["dist2goal"]
        _lib.check(_lib.load().dgppo_env_cfg_finalize(ctypes.byref(c)), "dgppo_env_cfg_finalize")
        return c

    def agent_candidates(self, device=None) -> torch.Tensor:
        device = device or self.device
        key = ("cand", str(device))
        if key not in self._dev_cache:
            n = self._num_agents
            self._dev_cache[key] = torch.tensor([[i * n + j for j in range(n)] for i in range(n)],
                                                dtype=torch.int32).to(device)
        return self._dev_cache[key]

    def _record_view(self, states, record):
        extra = states.dim() - 2 - (record.dim() - 2)  # e.g. (B, T) graph views over (B,) records
        if extra > 0:
            record = record.reshape(record.shape[:1] + (1,) * extra + record.shape[1:]).expand(
                tuple(states.shape[:-2]) + tuple(record.shape[1:]))
        return record

    def _assemble(self, nodes, edges, states, recv, send, obstacles) -> GraphsTuple:
        g = super()._assemble(nodes, edges, states, recv, send, obstacles)
        return g._replace(env_states=self._env_states(states, obstacles, nodes))

    def _obstacles_of(self, graph: GraphsTuple) -> torch.Tensor:
        rec = graph.env_states.record if graph.env_states is not None else None
        if rec is None:
            raise ValueError(f"{type(self).__name__} graph carries no env record (env_states.record is None)")
        if rec.stride(-1) != 1 or rec.stride(-2) != _lib.DGPPO_VMAS_FIELDS:
            raise ValueError("VMAS env records must be contiguous per env")
        return rec


class VMASWheel(VMASEnv):
    """vmas_wheel.py:35-307."""

    ENGINE = _lib.DGPPO_ENGINE_VMAS_WHEEL
    HALF_WIDTH = 1.2
    N_OBS = 0
    NODE_DIM = 13  # [pos(2), vel(2), line sincos(2), line angvel(1), contact_force(2), goal sincos(2), obs sincos(2)]

    def __init__(self, num_agents: int, area_size: Optional[float] = None, max_step: int = 64, dt: float = 0.1,
                 params: dict = None, device=None):
        super().__init__(num_agents, area_size, max_step, dt, params, device)
        self.line_length = 2.0
        self.obs_halfwidth_rad = float(torch.deg2rad(torch.tensor(15.0, dtype=torch.float64)))
        self.obs_init_pad_rad = float(torch.deg2rad(torch.tensor(1.0, dtype=torch.float64)))
        self.frame_skip = 3

    @property
    def cost_components(self) -> Tuple[str, ...]:
        return ("agent collisions",)

    def _env_states(self, states, obstacles, nodes=None):
        rec = self._record_view(states, obstacles) if obstacles is not None else None
        return VMASWheelState(states[..., 3, 0], states[..., 3, 1], states[..., :3, :2], states[..., :3, 2:4],
                              nodes[..., :3, 7:9] if nodes is not None else None,
                              rec[..., 0, 0] if rec is not None else None, rec[..., 0, 1] if rec is not None else None,
                              rec)


class VMASReverseTransport(VMASEnv):
    """vmas_reverse_transport.py:32-312."""

    ENGINE = _lib.DGPPO_ENGINE_VMAS_TRANSPORT
    HALF_WIDTH = 0.8
    N_OBS = 3
    NODE_DIM = 20  # [pos, vel, box_pos, box_vel, rel_goal_pos, in_contact, rel_obs_pos_vec(6), rel_obs_dist(3)]

    def __init__(self, num_agents: int, area_size: Optional[float] = None, max_step: int = 64, dt: float = 0.1,
                 params: dict = None, device=None):
        super().__init__(num_agents, area_size, max_step, dt, params, device)
        self.package_width = 0.6
        self.package_length = 0.6
        self.package_mass = 10.0
        self.obs_radius = 0.15
        self.frame_skip = 4

    @property
    def cost_components(self) -> Tuple[str, ...]:
        return "agent collisions", "obstacle collisions"

    def _env_states(self, states, obstacles, nodes=None):
        rec = self._record_view(states, obstacles) if obstacles is not None else None
        return VMASReverseTransportState(states[..., 3, :2], states[..., 3, 2:4], states[..., :3, :2],
                                         states[..., :3, 2:4], rec[..., 0, :2] if rec is not None else None,
                                         rec[..., 0, 2:].unflatten(-1, (3, 2)) if rec is not None else None, rec)


__all__ = ["VMASEnv", "VMASWheel", "VMASReverseTransport", "VMASWheelState", "VMASReverseTransportState"]

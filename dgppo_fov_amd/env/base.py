"""MultiAgentEnv: the reference's env plugin API (dgppo/env/base.py:30-150), batched over envs.

Differences from the reference, all deliberate:
  * `reset(key, n_env)` / `step(graph, action)` take and return env-batched tensors (leading B);
    the reference's per-env functions are `jax.vmap`-ed by the algorithm instead.
  * `step` runs ONE fused HIP kernel (dgppo_env_step in libdgppo_hip.so) that does dynamics,
    LiDAR, reward, cost and the padded graph build; `reset` runs dgppo_env_reset.
  * `PARAMS` is copied per instance (the reference mutates the class dict in make_env).
There is no CPU fallback: without the HIP library every call raises NativeLibraryError.
"""
from __future__ import annotations

import copy
import ctypes
from abc import ABC
from typing import NamedTuple, Optional, Tuple

import numpy as np
import torch

from .. import _lib, ops
from ..utils.graph import GraphsTuple


class StepResult(NamedTuple):
    graph: GraphsTuple
    reward: torch.Tensor  # (B,)
    cost: torch.Tensor  # (B, n, n_cost)
    done: torch.Tensor  # (B,) bool, always False (fixed-horizon episodes)
    info: dict


class RolloutResult(NamedTuple):
    Tp1_graph: GraphsTuple
    T_action: torch.Tensor
    T_reward: torch.Tensor
    T_cost: torch.Tensor
    T_done: torch.Tensor
    T_info: dict
    T_rnn_state: torch.Tensor


class MultiAgentEnv(ABC):
    PARAMS: dict = {}
    ENGINE: int = _lib.DGPPO_ENGINE_LIDAR
    GOAL_MODE: int = _lib.DGPPO_GOAL_SPREAD

    AGENT = 0
    GOAL = 1
    OBS = 2

    # node columns a never-receiving node can have nonzero (None: all); the GNN's agent-mode layers read only
    # these when the nodes are wider than the attention kernels' raw-row limit (nn/layers.py GraphBatch)
    nonagent_feature_cols = None

    def __init__(self, num_agents: int, area_size: float, max_step: int = 256, dt: float = 0.03,
                 params: Optional[dict] = None, device=None):
        self._num_agents = int(num_agents)
        self._dt = dt
        self._params = copy.deepcopy(self.PARAMS if params is None else params)
        self._t = 0
        self._max_step = max_step
        self._area_size = area_size
        self.num_goals = self._n_goals()  # goal node rows (the line / formation variants: landmarks)
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu"))
        self._cfg = self._make_cfg()
        self._cfg_handle = ops.register_env_cfg(self._cfg, owner=self)  # the torch.ops.dgppo env ops take this handle
        self._dev_cache = {}

    def _n_goals(self) -> int:
        return self._num_agents

    # ---- reference properties --------------------------------------------------------------
    @property
    def params(self) -> dict:
        return self._params

    @property
    def num_agents(self) -> int:
        return self._num_agents

    @property
    def area_size(self) -> float:
        return self._area_size

    @property
    def dt(self) -> float:
        return self._dt

    @property
    def max_episode_steps(self) -> int:
        return self._max_step

    @property
    def n_cost(self) -> int:
        return 2

    @property
    def cost_components(self) -> Tuple[str, ...]:
        return "agent collisions", "obs collisions"

    @property
    def state_dim(self) -> int:
        return 4

    @property
    def node_dim(self) -> int:
        return self.state_dim + 3

    @property
    def edge_dim(self) -> int:
        return 4

    @property
    def action_dim(self) -> int:
        return 2

    def state_lim(self, state=None):
        raise NotImplementedError

    def action_lim(self):
        return -torch.ones(self.action_dim), torch.ones(self.action_dim)

    def clip_state(self, state: torch.Tensor) -> torch.Tensor:
        lo, hi = self.state_lim(state)
        return torch.minimum(torch.maximum(state, lo.to(state)), hi.to(state))

    def clip_action(self, action: torch.Tensor) -> torch.Tensor:
        lo, hi = self.action_lim()
        return torch.minimum(torch.maximum(action, lo.to(action)), hi.to(action))

    # ---- graph geometry --------------------------------------------------------------------
    @property
    def n_obs(self) -> int:
        return int(self._params["n_obs"])

    @property
    def n_nodes(self) -> int:
        return int(self._cfg.n_nodes)

    @property
    def n_edges(self) -> int:
        return int(self._cfg.n_edges)

    @property
    def cfg(self) -> _lib.EnvCfg:
        return self._cfg

    def _obstacle_fields(self) -> int:
        return 0

    def _obstacle_rows(self) -> int:
        """Rows of the per-env obstacle buffer (env_states records the step kernels read)."""
        return max(self.n_obs, 1)

    def _make_cfg(self) -> _lib.EnvCfg:
        p = self._params
        c = _lib.EnvCfg()
        c.engine = self.ENGINE
        c.goal_mode = self.GOAL_MODE
        c.n_agents = self._num_agents
        c.n_obs = int(p["n_obs"])
        c.n_rays = int(p.get("n_rays", 0))
        c.top_k = int(p.get("top_k_rays", 0))
        c.state_dim = self.state_dim
        c.node_dim = self.node_dim
        c.dt = self._dt
        c.comm_radius = p["comm_radius"]
        c.car_radius = p["car_radius"]
        c.obs_radius = p.get("obs_radius", 0.0)
        c.area_size = self._area_size
        c.dist2goal = p["dist2goal"]
        lo, hi = p.get("obs_len_range", [0.1, 0.3])
        c.obs_len_lo, c.obs_len_hi = lo, hi
        c.obs_theta_lo, c.obs_theta_hi = self._obs_theta_range()
        # derived constants in Python float64 arithmetic, rounded once (as the reference does)
        r, cr = p["car_radius"], p["comm_radius"]
        orr = p.get("obs_radius", 0.0)
        mpe = self.ENGINE == _lib.DGPPO_ENGINE_MPE
        c.c_agent_cost = r * 2
        c.c_obs_cost = (r + orr) if mpe else r
        c.c_self_dist = cr + 1
        c.c_lidar_active = cr - 1e-1
        md = 2 * r if mpe else 2.2 * r
        c.c_min_dist = md
        c.c_inside_r = md / 2
        c.c_mpe_obs_agent = r + orr
        c.c_mpe_obs_goal = r * 2 + orr
        c.c_mpe_obs_lo = r * 3
        c.c_mpe_obs_hi = self._area_size - r * 3
        c.n_goals = self.num_goals if self.num_goals != self._num_agents else 0
        self._engine_cfg(c)
        _lib.check(_lib.load().dgppo_env_cfg_finalize(ctypes.byref(c)), "dgppo_env_cfg_finalize")
        return c

    def _engine_cfg(self, c: _lib.EnvCfg) -> None:
        """Engine-specific cfg fields (hook for subclasses), set before dgppo_env_cfg_finalize."""

    def _obs_theta_range(self):
        return 0.0, 2 * np.pi

    # ---- device constants -------------------------------------------------------------------
    def _ray_table(self, device):
        key = ("rays", str(device))
        if key not in self._dev_cache:
            self._dev_cache[key] = ray_table(int(self._params.get("n_rays", 1) or 1),
                                             float(self._params["comm_radius"])).to(device)
        return self._dev_cache[key]

    def _count_scalars(self, device):
        key = ("counts", str(device))
        if key not in self._dev_cache:  # built once: no per-step fill kernels in a captured rollout
            self._dev_cache[key] = (torch.tensor(self.n_nodes, dtype=torch.int32, device=device),
                                    torch.tensor(self.n_edges, dtype=torch.int32, device=device))
        return self._dev_cache[key]

    def node_type_row(self, device=None) -> torch.Tensor:
        device = device or self.device
        key = ("node_type", str(device))
        if key not in self._dev_cache:
            n, ng, N = self._num_agents, self.num_goals, self.n_nodes
            t = -torch.ones(N, dtype=torch.int32)
            t[:n] = self.AGENT
            t[n:n + ng] = self.GOAL
            t[n + ng:N - 1] = self.OBS
            self._dev_cache[key] = t.to(device)
        return self._dev_cache[key]

    def agent_candidates(self, device=None) -> torch.Tensor:
        """(n, C) int32: for each agent i, the edge ids of the padded layout whose receiver may be i
        (agent-agent row i, its goal edge(s), its lidar hits / obstacle edges).  The GNN kernels
        keep a candidate iff receivers[e] == i at run time (masked edges point at the pad node)."""
        device = device or self.device
        key = ("cand", str(device))
        if key not in self._dev_cache:
            n, ng = self._num_agents, self.num_goals
            spread = self.GOAL_MODE == _lib.DGPPO_GOAL_SPREAD
            n_ag = n * ng if spread else n
            mpe = self.ENGINE == _lib.DGPPO_ENGINE_MPE
            k = self.n_obs if mpe else (int(self._params.get("top_k_rays", 0)) if self.n_obs > 0 else 0)
            rows = []
            for i in range(n):
                r = [i * n + j for j in range(n)]
                r += [n * n + i * ng + j for j in range(ng)] if spread else [n * n + i]
                r += [n * n + n_ag + i * k + h for h in range(k)]
                rows.append(r)
            self._dev_cache[key] = torch.tensor(rows, dtype=torch.int32).to(device)
        return self._dev_cache[key]

    # ---- buffers ----------------------------------------------------------------------------
    def empty_graph(self, batch_shape, device=None) -> GraphsTuple:
        """Allocate an uninitialised batched graph (the kernel fills every element)."""
        device = device or self.device
        bs = tuple(batch_shape) if isinstance(batch_shape, (tuple, list)) else (int(batch_shape),)
        N, E = self.n_nodes, self.n_edges
        f32 = dict(dtype=torch.float32, device=device)
        i32 = dict(dtype=torch.int32, device=device)
        nodes = torch.empty(bs + (N, self.node_dim), **f32)
        states = torch.empty(bs + (N, self.state_dim), **f32)
        edges = torch.empty(bs + (E, self.edge_dim), **f32)
        recv = torch.empty(bs + (E,), **i32)
        send = torch.empty(bs + (E,), **i32)
        return self._assemble(nodes, edges, states, recv, send, None)

    def _assemble(self, nodes, edges, states, recv, send, obstacles) -> GraphsTuple:
        bs = tuple(nodes.shape[:-2])
        dev = nodes.device
        n_node, n_edge = self._count_scalars(dev)
        n_node, n_edge = n_node.expand(bs), n_edge.expand(bs)
        node_type = self.node_type_row(dev).expand(bs + (self.n_nodes,))
        env_states = self._env_states(states, obstacles)
        return GraphsTuple(n_node, n_edge, nodes, edges, states, recv, send, node_type, env_states)

    def _env_states(self, states, obstacles):
        raise NotImplementedError

    @staticmethod
    def _env_stride(t: torch.Tensor, inner: int) -> int:
        """Per-env element stride of t, requiring the trailing `inner` elements to be contiguous."""
        tail = 1
        for d in range(t.dim() - 1, t.dim() - 1 - inner, -1):
            if t.stride(d) != tail:
                raise ValueError("trailing dims must be contiguous")
            tail *= t.shape[d]
        return t.stride(t.dim() - 1 - inner) if t.dim() > inner else tail

    # ---- reset / step ------------------------------------------------------------------------
    def reset(self, key=0, n_env: int = 1, env_offset: int = 0, out: Optional[GraphsTuple] = None,
              obstacles_out: Optional[torch.Tensor] = None) -> GraphsTuple:
        """Batched `vmap(env.reset)`: env b samples from Philox keyed (key, env_offset + b).

        `key` is an int, or a 1-element uint64/int64 device tensor read by the kernel at run time
        (so a captured hipGraph can be replayed with fresh keys)."""
        dev = self.device if out is None else out.nodes.device
        _lib.require_gpu(dev, "env.reset")
        g = self.empty_graph((n_env,), dev) if out is None else out
        ob = obstacles_out
        if ob is None and self._obstacle_fields() > 0:
            ob = torch.empty((n_env, self._obstacle_rows(), self._obstacle_fields()), dtype=torch.float32, device=dev)
        tkey = key if isinstance(key, torch.Tensor) else None
        seed = 0 if tkey is not None else int(key) & 0xFFFFFFFFFFFFFFFF
        torch.ops.dgppo.env_reset(self._cfg_handle, tkey, seed if seed < 2 ** 63 else seed - 2 ** 64,
                                  int(env_offset), int(n_env), ob, self._ray_table(dev), g.nodes, g.edges, g.states,
                                  g.receivers, g.senders)
        return self._assemble(g.nodes, g.edges, g.states, g.receivers, g.senders, ob)

    def reset_states(self, key, n_env: int, env_offset: int = 0, out: Optional[GraphsTuple] = None,
                     obstacles_out: Optional[torch.Tensor] = None) -> GraphsTuple:
        """The sampling half of `reset` (torch.ops.dgppo.env_reset_states): obstacles and the agent / goal
        state rows only; `rollout_into(..., rebuild_first=True)` builds graph 0 from them.  Configs
        without the persistent rollout kernel get the full reset."""
        dev = self.device if out is None else out.nodes.device
        _lib.require_gpu(dev, "env.reset_states")
        g = self.empty_graph((n_env,), dev) if out is None else out
        ob = obstacles_out
        if ob is None and self._obstacle_fields() > 0:
            ob = torch.empty((n_env, self._obstacle_rows(), self._obstacle_fields()), dtype=torch.float32, device=dev)
        tkey = key if isinstance(key, torch.Tensor) else None
        seed = 0 if tkey is not None else int(key) & 0xFFFFFFFFFFFFFFFF
        torch.ops.dgppo.env_reset_states(self._cfg_handle, tkey, seed if seed < 2 ** 63 else seed - 2 ** 64,
                                         int(env_offset), int(n_env), ob, self._ray_table(dev), g.nodes, g.edges,
                                         g.states, g.receivers, g.senders)
        return self._assemble(g.nodes, g.edges, g.states, g.receivers, g.senders, ob)

    def rollout_into(self, buf: GraphsTuple, obstacles: Optional[torch.Tensor], actions: torch.Tensor,
                     rewards: torch.Tensor, costs: torch.Tensor, rebuild_first: bool = False) -> None:
        """T env steps with the given actions (T, B, n, A) in one call (torch.ops.dgppo.env_rollout): buf is
        a time-major (T+1, B, ...) graph buffer, step t reads buf[t] and writes buf[t+1], rewards[t],
        costs[t] -- the env half of the reference's rollout scan (trainer/utils.py:45-55)."""
        _lib.require_gpu(buf.states.device, "env.rollout")
        n, A = self._num_agents, self.action_dim
        T = actions.shape[0]
        if actions.shape[-2:] != (n, A) or buf.states.shape[0] != T + 1 or buf.states.dim() != 4:
            raise ValueError("rollout_into: actions (T, B, n, A) and a (T+1, B, N, sd) graph buffer")
        torch.ops.dgppo.env_rollout(self._cfg_handle, bool(rebuild_first), obstacles, actions,
                                    self._ray_table(buf.states.device), buf.nodes, buf.edges, buf.states,
                                    buf.receivers, buf.senders, rewards, costs)

    def step_into(self, graph: GraphsTuple, action: torch.Tensor, out: GraphsTuple,
                  reward: torch.Tensor, cost: torch.Tensor) -> GraphsTuple:
        """One fused HIP step (torch.ops.dgppo.env_step) writing into caller-owned buffers (views into a
        rollout buffer)."""
        _lib.require_gpu(graph.states.device, "env.step")
        if graph.states.dim() != 3:
            raise ValueError("step expects one leading env axis: states (B, N, state_dim)")
        B = graph.states.shape[0]
        n = self._num_agents
        if action.shape[-2:] != (n, self.action_dim):
            raise ValueError(f"action must be (B, {n}, {self.action_dim}), got {tuple(action.shape)}")
        if graph.states.shape[-2:] != (self.n_nodes, self.state_dim):
            raise ValueError("graph does not match this env's layout")
        if action.dtype != torch.float32:
            action = action.float()
        A = self.action_dim
        action = action if action.stride(-1) == 1 and action.stride(-2) == A else action.contiguous()
        ob = self._obstacles_of(graph)
        torch.ops.dgppo.env_step(self._cfg_handle, graph.states, ob, action, self._ray_table(graph.states.device),
                                 out.nodes, out.edges, out.states, out.receivers, out.senders, reward, cost)
        return self._assemble(out.nodes, out.edges, out.states, out.receivers, out.senders, ob)

    def _obstacles_of(self, graph: GraphsTuple) -> Optional[torch.Tensor]:
        return None

    def step(self, graph: GraphsTuple, action: torch.Tensor, get_eval_info: bool = False) -> StepResult:
        """Batched `vmap(env.step)` (lidar_env/base.py:151-174, mpe/base.py:137-158)."""
        B = graph.states.shape[:-2]
        out = self.empty_graph(B, graph.states.device)
        reward = torch.empty(B, dtype=torch.float32, device=graph.states.device)
        cost = torch.empty(B + (self._num_agents, self.n_cost), dtype=torch.float32, device=graph.states.device)
        g = self.step_into(graph, action, out, reward, cost)
        done = torch.zeros(B, dtype=torch.bool, device=graph.states.device)
        return StepResult(g, reward, cost, done, {})

    def get_cost(self, graph: GraphsTuple) -> torch.Tensor:
        """Cost of a graph (lidar_env/base.py:180-207): the step kernel evaluates it on its input."""
        zero = torch.zeros(graph.states.shape[:-2] + (self._num_agents, self.action_dim), device=graph.states.device)
        return self.step(graph, zero).cost


def ray_table(n_rays: int, sense_range: float) -> torch.Tensor:
    """(R, 2) per-ray end offsets (cos th * range, sin th * range) with th = jnp.linspace(-pi,
    pi - 2pi/R, R) (env/utils.py:51-55), computed by dgppo_ray_table in the native library."""
    out = torch.empty((n_rays, 2), dtype=torch.float32)
    _lib.check(_lib.load().dgppo_ray_table(int(n_rays), float(sense_range), ctypes.c_void_p(out.data_ptr())),
               "dgppo_ray_table")
    return out

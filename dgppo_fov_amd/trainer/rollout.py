"""Device-resident rollout driver: the reference's `rollout` / `test_rollout`
(dgppo/trainer/utils.py:22-86: reset, then lax.scan of (actor, env.step) over T steps) as a
fixed sequence of HIP launches over preallocated (B, T+1, ...) HBM buffers, optionally captured
once into a hipGraph and replayed (one host call per episode instead of 2T+1 launches).

The actor is any callable `actor(graph_t, t)` that writes actions into `self.actions[:, t]`
(and log-probs / carries into its own buffers) with device-side launches only; `None` keeps the
actions already stored in `self.actions` (synthetic/random-action rollouts)."""
from __future__ import annotations

from typing import Callable, Optional

import torch

from ..env.base import MultiAgentEnv
from ..utils.graph import GraphsTuple
from .data import Rollout


class RolloutEngine:
    def __init__(self, env: MultiAgentEnv, n_env: int, T: Optional[int] = None, device=None, env_offset: int = 0,
                 actor: Optional[Callable] = None):
        self.env = env
        self.B = int(n_env)
        self.T = int(T or env.max_episode_steps)
        self.device = torch.device(device) if device is not None else env.device
        self.env_offset = int(env_offset)
        self.actor = actor
        B, T, n = self.B, self.T, env.num_agents
        self.buf = env.empty_graph((B, T + 1), self.device)
        nf = env._obstacle_fields()
        self.obstacles = (torch.empty((B, max(env.n_obs, 1), nf), dtype=torch.float32, device=self.device)
                          if nf else None)
        self.actions = torch.zeros((B, T, n, env.action_dim), dtype=torch.float32, device=self.device)
        self.rewards = torch.empty((B, T), dtype=torch.float32, device=self.device)
        self.costs = torch.empty((B, T, n, env.n_cost), dtype=torch.float32, device=self.device)
        self.dones = torch.zeros((B, T), dtype=torch.bool, device=self.device)
        self.key = torch.zeros(1, dtype=torch.int64, device=self.device)
        self._hip_graph = None

    def graph_at(self, t: int) -> GraphsTuple:
        b = self.buf
        return self.env._assemble(b.nodes[:, t], b.edges[:, t], b.states[:, t], b.receivers[:, t],
                                  b.senders[:, t], self.obstacles)

    def _run(self):
        env = self.env
        cur = env.reset(self.key, n_env=self.B, env_offset=self.env_offset, out=self.graph_at(0),
                        obstacles_out=self.obstacles)
        for t in range(self.T):
            if self.actor is not None:
                self.actor(cur, t)
            cur = env.step_into(cur, self.actions[:, t], self.graph_at(t + 1), self.rewards[:, t], self.costs[:, t])

    def capture(self):
        """Record reset + T steps into one hipGraph (after one eager warm-up run)."""
        self._run()
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._run()
        self._hip_graph = g
        return self

    def run(self, key: int) -> Rollout:
        self.key.fill_(int(key))
        if self._hip_graph is not None:
            self._hip_graph.replay()
        else:
            self._run()
        return self.rollout()

    def rollout(self) -> Rollout:
        b = self.buf
        T = self.T

        def view(sl):
            return self.env._assemble(b.nodes[:, sl], b.edges[:, sl], b.states[:, sl], b.receivers[:, sl],
                                      b.senders[:, sl], self.obstacles)

        return Rollout(view(slice(0, T)), self.actions, None, self.rewards, self.costs, self.dones, None,
                       view(slice(1, T + 1)))

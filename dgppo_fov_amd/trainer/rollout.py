"""Device-resident rollout driver: the reference's `rollout` / `test_rollout`
(dgppo/trainer/utils.py:22-86: reset, then lax.scan of (actor, env.step) over T steps) as a fixed
sequence of HIP launches over preallocated TIME-MAJOR HBM buffers, optionally captured once into
a hipGraph and replayed (one host call per episode instead of ~25T launches).

Buffers are time-major, (T+1, B, ...), so the graph of step t is one contiguous (B, ...) block
that the env-step and GNN kernels read and write without copies; the Rollout handed to the
algorithm exposes the reference's (B, T, ...) leading dims as permuted views.

Actor carry semantics follow the reference exactly:
  stochastic `rollout`   rnn_states[t] = carry BEFORE acting on graph t (utils.py:186-192)
  deterministic `test_rollout` rnn_states[t] = carry AFTER acting on graph t (utils.py:211-218)
"""
from __future__ import annotations

from typing import Optional

import ctypes

import torch

from .. import _lib
from ..env.base import MultiAgentEnv
from ..nn import kernels as K
from ..nn.layers import GraphBatch
from ..utils.graph import GraphsTuple
from .data import Rollout


class RolloutEngine:
    MODE_RANDOM, MODE_SAMPLE, MODE_DET = -1, 1, 0

    def __init__(self, env: MultiAgentEnv, n_env: int, T: Optional[int] = None, device=None, env_offset: int = 0,
                 actor=None, mode: int = -1, lanes: int = 1, fused: bool = True):
        """actor: an ActorNet (or None); mode: MODE_SAMPLE (stochastic policy, sample_action),
        MODE_DET (deterministic policy, get_action) or MODE_RANDOM (keep `self.actions` as given).
        lanes: split the envs into that many contiguous slices, each running its T (act, step) pairs
        on its own HIP stream after the shared reset, so one slice's launch ramp and store drain
        overlap the other's compute (envs are independent: results are identical).  With an actor
        this needs the fused policy step (it reads only the prepared query-key workspace); the T
        sampling-noise tensors are drawn up front with the same Philox stream ids.
        fused: an env-only (MODE_RANDOM, one lane) rollout runs as a states-only reset plus one persistent
        dgppo_env_rollout launch for all T steps (else reset + T step launches; identical results)."""
        self.env = env
        self.B = int(n_env)
        self.T = int(T or env.max_episode_steps)
        self.device = torch.device(device) if device is not None else env.device
        self.env_offset = int(env_offset)
        self.actor = actor
        self.mode = mode if actor is not None else self.MODE_RANDOM
        B, T, n, dev = self.B, self.T, env.num_agents, self.device
        self.buf = env.empty_graph((T + 1, B), dev)
        nf = env._obstacle_fields()
        self.obstacles = (torch.empty((B, env._obstacle_rows(), nf), dtype=torch.float32, device=dev) if nf else None)
        self.actions = torch.zeros((T, B, n, env.action_dim), dtype=torch.float32, device=dev)
        self.rewards = torch.empty((T, B), dtype=torch.float32, device=dev)
        self.costs = torch.empty((T, B, n, env.n_cost), dtype=torch.float32, device=dev)
        self.dones = torch.zeros((T, B), dtype=torch.bool, device=dev)
        self.key = torch.zeros(1, dtype=torch.int64, device=dev)
        if actor is not None:
            self.W = actor.carry_width  # carry floats per agent: (rnn_layers, carries, 64) flattened
            self.rnn = torch.zeros((T + 1, B, n, self.W), dtype=torch.float32, device=dev)
            self.log_pis = torch.zeros((T, B, n), dtype=torch.float32, device=dev)
            self.noise = torch.empty((B * n, env.action_dim), dtype=torch.float32, device=dev)
        self._hip_graph = None
        self.fused = bool(fused)
        self.lanes = int(lanes)
        if self.lanes > 1 and B % self.lanes:
            raise ValueError(f"n_env {B} is not a multiple of lanes {self.lanes}")
        if self.lanes > 1 and actor is not None and actor._fused_args(self._batch(0)) is None:
            self.lanes = 1  # the unfused actor path shares GEMM workspaces: one stream only
        if self.lanes > 1:
            self._streams = [torch.cuda.Stream(dev) for _ in range(self.lanes)]
            if self.mode == self.MODE_SAMPLE:
                self.noise_all = torch.empty((T, B * n, env.action_dim), dtype=torch.float32, device=dev)

    def graph_at(self, t: int) -> GraphsTuple:
        b = self.buf
        return self.env._assemble(b.nodes[t], b.edges[t], b.states[t], b.receivers[t], b.senders[t], self.obstacles)

    def _batch(self, t: int, sl=slice(None)) -> GraphBatch:
        env, b = self.env, self.buf
        return GraphBatch(b.nodes[t][sl], b.edges[t][sl], b.receivers[t][sl], b.senders[t][sl], env.num_agents,
                          env.agent_candidates(self.device), raw_cols=env.nonagent_feature_cols)

    def _act_slice(self, t: int, sl: slice, k: int):
        n, A, w = self.env.num_agents, self.env.action_dim, sl.stop - sl.start
        h = self.rnn[t][sl].view(w * n, self.W)
        kw = dict(action_out=self.actions[t][sl].view(-1, A), h_out=self.rnn[t + 1][sl].view(w * n, self.W), prepare=False)
        if self.mode == self.MODE_SAMPLE:
            self.actor.act(self._batch(t, sl), h, 1, noise=self.noise_all[t][k * w * n:(k + 1) * w * n],
                           log_pi_out=self.log_pis[t][sl].view(-1), **kw)
        else:
            self.actor.act(self._batch(t, sl), h, 0, **kw)

    def _act(self, t: int):
        env = self.env
        g = self._batch(t)
        n = env.num_agents
        h = self.rnn[t].view(self.B * n, self.W)
        if self.mode == self.MODE_SAMPLE:
            # per-step, per-shard Philox stream (env_offset, t) -> disjoint noise across ranks, drawn inside the
            # fused policy step (K.normal_ into self.noise first on the unfused path)
            self.actor.act(g, h, 1, noise=self.noise, action_out=self.actions[t].view(-1, env.action_dim),
                           log_pi_out=self.log_pis[t].view(-1), h_out=self.rnn[t + 1].view(self.B * n, self.W),
                           prepare=t == 0, noise_seed=self.key, noise_stream=(self.env_offset << 32) | t)
        else:
            self.actor.act(g, h, 0, action_out=self.actions[t].view(-1, env.action_dim),
                           h_out=self.rnn[t + 1].view(self.B * n, self.W), prepare=t == 0)

    def _run(self):
        env = self.env
        if self.mode == self.MODE_RANDOM and self.lanes == 1 and self.fused:
            # env-only rollout: the states-only reset + ONE persistent launch for all T steps (graph 0 built
            # by the rollout kernel; configs without it loop the step kernel inside the call)
            env.reset_states(self.key, n_env=self.B, env_offset=self.env_offset, out=self.graph_at(0),
                             obstacles_out=self.obstacles)
            env.rollout_into(self.buf, self.obstacles, self.actions, self.rewards, self.costs, rebuild_first=True)
            return
        cur = env.reset(self.key, n_env=self.B, env_offset=self.env_offset, out=self.graph_at(0),
                        obstacles_out=self.obstacles)
        if self.lanes > 1:
            self._run_lanes()
            return
        for t in range(self.T):
            if self.mode != self.MODE_RANDOM:
                self._act(t)
            cur = env.step_into(cur, self.actions[t], self.graph_at(t + 1), self.rewards[t], self.costs[t])

    def _run_lanes(self):
        env, b, main = self.env, self.buf, torch.cuda.current_stream(self.device)
        w = self.B // self.lanes
        if self.actor is not None:
            fa = self.actor._fused_args(self._batch(0))  # not None: checked in __init__
            K._chk(_lib.load().dgppo_policy_prepare(ctypes.byref(fa), _lib.stream_handle(self.device)),
                   "dgppo_policy_prepare")
            if self.mode == self.MODE_SAMPLE:
                for t in range(self.T):
                    K.normal_(self.noise_all[t], stream_id=(self.env_offset << 32) | t, seed_tensor=self.key)
        for k, s in enumerate(self._streams):
            sl = slice(k * w, (k + 1) * w)
            obst = self.obstacles[sl] if self.obstacles is not None else None
            at = lambda t: env._assemble(b.nodes[t][sl], b.edges[t][sl], b.states[t][sl],  # noqa: E731
                                         b.receivers[t][sl], b.senders[t][sl], obst)
            s.wait_stream(main)
            with torch.cuda.stream(s):
                cur = at(0)
                for t in range(self.T):
                    if self.actor is not None:
                        self._act_slice(t, sl, k)
                    cur = env.step_into(cur, self.actions[t][sl], at(t + 1), self.rewards[t][sl], self.costs[t][sl])
        for s in self._streams:
            main.wait_stream(s)

    def capture(self):
        """Record reset + T x (actor, step) into one hipGraph (after one eager warm-up run)."""
        self._run()
        torch.cuda.synchronize(self.device)
        g = K.hold_for_graph(torch.cuda.CUDAGraph())
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
        """(B, T, ...) views of the time-major buffers (Rollout of dgppo/trainer/data.py)."""
        b, T = self.buf, self.T

        def view(sl):
            tr = lambda x: x[sl].transpose(0, 1)  # noqa: E731
            return self.env._assemble(tr(b.nodes), tr(b.edges), tr(b.states), tr(b.receivers), tr(b.senders),
                                      self.obstacles)

        rnn = None
        log_pis = None
        if self.actor is not None:
            # (B, T, rnn_layers, n, carries, 64): rnn_states[t] = carry before (stochastic) / after (deterministic)
            # step t; a view of the (T+1, B, n, W) buffer
            sl = slice(0, T) if self.mode == self.MODE_SAMPLE else slice(1, T + 1)
            rs = self.actor.gru
            rnn = self.rnn[sl].transpose(0, 1).unflatten(-1, (rs.layers, rs.carries, 64)).movedim(-4, -3)
            log_pis = self.log_pis.transpose(0, 1) if self.mode == self.MODE_SAMPLE else None
        return Rollout(view(slice(0, T)), self.actions.transpose(0, 1), rnn, self.rewards.transpose(0, 1),
                       self.costs.transpose(0, 1), self.dones.transpose(0, 1), log_pis, view(slice(1, T + 1)))

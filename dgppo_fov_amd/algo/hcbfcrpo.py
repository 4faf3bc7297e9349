"""HCBF-CRPO (dgppo/algo/hcbfcrpo.py): DGPPO with a hand-crafted CBF — Vh is the env's own cost of each
graph (`get_Vh = env.get_cost`, hcbfcrpo.py:96-99), so there is no Vh network and no deterministic
rollout: Vh[:, :T] = the rollout's pre-step costs, Vh[:, T] = the cost of the last next-graph
(hcbfcrpo.py:145-155); Dec-OCP GAE on (costs, -reward); DGPPO's merged CBF advantage
(dgppo_advantages, hcbfcrpo.py:163-183); per minibatch update_Vl and update_policy.
"""
from __future__ import annotations

import torch

from ..nn import kernels as K
from ..trainer.rollout import Rollout
from .informarl import InforMARL


class HCBFCRPO(InforMARL):
    @property
    def config(self) -> dict:
        c = dict(super(InforMARL, self).config)
        c.pop("Vh_gnn_layers", None)
        c.pop("lr_Vh", None)
        return c

    def _final_cost(self, rollout: Rollout) -> torch.Tensor:
        """env.get_cost of next_graph[:, -1] (B, n, n_cost)."""
        ng = rollout.next_graph
        ob = getattr(ng.env_states, "obstacle", None)
        ob = ob.packed[:, -1].contiguous() if ob is not None and hasattr(ob, "packed") else None
        g = self._env._assemble(ng.nodes[:, -1].contiguous(), ng.edges[:, -1].contiguous(), ng.states[:, -1].contiguous(),
                                ng.receivers[:, -1].contiguous(), ng.senders[:, -1].contiguous(), ob)
        return self._env.get_cost(g)

    def _targets(self, rollout: Rollout, Vl: torch.Tensor, step: int):
        env, dev = self._env, self.device
        B, T = rollout.rewards.shape
        n = self._n_agents
        costs = rollout.costs.contiguous()
        Vh = torch.empty((B, T + 1, n, env.n_cost), device=dev)
        Vh[:, :T].copy_(costs)
        Vh[:, T].copy_(self._final_cost(rollout))
        Qh = torch.empty((B, T, n, env.n_cost), device=dev)
        Ql = torch.empty((B, T), device=dev)
        K.gae(costs, (-rollout.rewards).contiguous(), Vh, Vl, Qh, Ql, self.gamma, self.gae_lambda)
        A = torch.empty((B, T, n), device=dev)
        safe_cnt = torch.empty(B, device=dev)
        K.dgppo_advantages(Ql, Vl, Vh, A, safe_cnt, env.dt, self.alpha, self.cbf_eps, self.cbf_weight_at(step))
        if self.trace is not None:
            self.trace.update(Vl=Vl.clone(), Vh=Vh.clone(), Ql=Ql.clone(), A=A.clone())
        safe = safe_cnt.sum()
        if self.world > 1:
            torch.distributed.all_reduce(safe)
        return Ql, A, {"eval/safe_data": safe / (B * self.world * T * n)}

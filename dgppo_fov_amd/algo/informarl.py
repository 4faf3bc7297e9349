"""InforMARL (dgppo/algo/informarl.py): the GNN PPO baseline DGPPO extends — policy + Vl only, the
costs entering the GAE loss with weight `cost_weight` (informarl.py:318-340):

  l = -reward + w * sum_a sum_h max(cost, 0),  w = cost_weight (x5 at 50% and x5 at 75% of train_steps
  when cost_schedule, informarl.py:189-198);
  (Qh, Ql) = compute_dec_ocp_gae(costs, l, Vh = Vl broadcast, Vl);  Al = Ql - Vl;
  A = -(Al - mean_t Al) / (std_t Al + 1e-8) for every agent;
  per minibatch: update_Vl (l2 to Ql) and update_policy (clipped PPO + entropy), clip + Adam each.

Same kernels as DGPPO (GNN / GRU / TanhNormal / GAE / losses / Adam) plus dgppo_cost_shaped_loss and
dgppo_informarl_advantages.  The Vh network DGPPO builds is allocated but never used or stepped.
"""
from __future__ import annotations

import torch

from ..nn import kernels as K
from ..trainer.rollout import Rollout
from .dgppo import PREPASS_GRAPHS, DGPPO, minibatch_plan


class InforMARL(DGPPO):
    def __init__(self, *args, cost_weight: float = 0.0, cost_schedule: bool = False, **kwargs):
        super().__init__(*args, **kwargs)
        self.cost_weight, self.cost_schedule = float(cost_weight), bool(cost_schedule)

    @property
    def config(self) -> dict:
        c = dict(super().config)
        c.update(cost_weight=self.cost_weight, cost_schedule=self.cost_schedule)
        for k in ("alpha", "cbf_eps", "cbf_weight", "cbf_schedule", "Vh_gnn_layers", "lr_Vh"):
            c.pop(k, None)
        return c

    def cost_weight_at(self, step: int) -> float:
        """optax.piecewise_constant_schedule(cost_weight, {0.5 T: 5, 0.75 T: 5}) (informarl.py:189-198)."""
        w = self.cost_weight
        if self.cost_schedule:
            if step >= int(self.train_steps * 0.5):
                w *= 5
            if step >= int(self.train_steps * 0.75):
                w *= 5
        return w

    def _targets(self, rollout: Rollout, Vl: torch.Tensor, step: int):
        """GAE on the cost-shaped loss with Vh = Vl broadcast, normalised advantages (informarl.py:324-340).
        Returns Ql (B, T), A (B, T, n) and extra info entries."""
        env, dev = self._env, self.device
        B, T = rollout.rewards.shape
        n = self._n_agents
        costs = rollout.costs.contiguous()
        l = torch.empty((B, T), device=dev)
        K.cost_shaped_loss(rollout.rewards.contiguous(), costs, self.cost_weight_at(step), l)
        Vh = Vl[:, :, None, None].expand(B, T + 1, n, env.n_cost).contiguous()
        Qh = torch.empty((B, T, n, env.n_cost), device=dev)
        Ql = torch.empty((B, T), device=dev)
        K.gae(costs, l, Vh, Vl, Qh, Ql, self.gamma, self.gae_lambda)
        A = torch.empty((B, T, n), device=dev)
        K.informarl_advantages(Ql, Vl, A)
        if self.trace is not None:
            self.trace.update(Vl=Vl.clone(), l=l.clone(), Ql=Ql.clone(), A=A.clone())
        return Ql, A, {}

    def update(self, rollout: Rollout, step: int) -> dict:
        dev = self.device
        B, T = rollout.rewards.shape
        chunk = max(1, min(B, PREPASS_GRAPHS // T))
        info, extra = {}, {}
        for _ in range(self.epoch_ppo):
            # Vl scan over the whole episode + final Vl (informarl.py:310-322)
            Vl = self._vl_all(rollout, chunk)
            Ql, A, extra = self._targets(rollout, Vl, step)
            # minibatches (informarl.py:342-355)
            L = self.rnn_step
            assert T % L == 0, "jnp.array(jnp.array_split(...)) in the reference needs rnn_step | T"
            S_per_env = T // L
            batches = minibatch_plan(B, T, self.world, self.batch_size, self.np_rng)
            env_ids = self._env_ids(batches)
            for bi in batches:
                envs = next(env_ids)
                Bm = len(bi)
                self.grad_flat.zero_()
                rg = rollout.graph
                nodes, edges, recv, send, acts, lp_old, adv, tgt = self._gather(
                    envs, rg.nodes, rg.edges, rg.receivers, rg.senders, rollout.actions, rollout.log_pis, A, Ql)
                g = self._graph_batch(nodes, edges, recv, send)
                v, _, cache = self.Vl.seq_fwd(g, Bm * S_per_env, L)
                tgt = tgt.view(Bm * S_per_env, L)
                dv = torch.empty_like(v)
                vl_loss = torch.empty(1, device=dev)
                K.l2_loss(v, tgt, dv, vl_loss)
                self.Vl.seq_bwd(cache, dv)
                del cache
                acts, lp_old, adv = acts.view(-1, self._action_dim), lp_old.view(-1), adv.view(-1)
                lp, ent, cache = self.actor.eval_seq_fwd(g, Bm * S_per_env, L, acts, self.entropy_eps)
                dlp = torch.empty_like(lp)
                dent = torch.empty_like(ent)
                stats = torch.empty(4, device=dev)
                K.ppo_loss(lp, lp_old, adv, ent, self.clip_eps, self.coef_ent, dlp, dent, stats)
                self.actor.eval_seq_bwd(cache, dlp, dent)
                del cache
                self._allreduce_grads()
                if self.trace is not None:
                    self.trace.setdefault("mb", []).append(dict(envs=bi.copy(), grad=self.grad_flat.clone()))
                for name in ("Vl", "policy"):
                    self.opt[name].step()
                info = {"Vl/loss": vl_loss, "Vl/max_target": tgt.max(), "Vl/min_target": tgt.min(),
                        "policy/stats": stats, "policy/log_pi_min": lp_old.min()}
        info.update(extra)
        out = self._finish_info(info)
        for k in ("Vh/grad_Vh_norm", "Vh/grad_Vh_has_nan"):
            out.pop(k, None)
        return out

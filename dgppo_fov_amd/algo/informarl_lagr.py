"""InforMARL-Lagr (dgppo/algo/informarl_lagr.py:25-327): InforMARL with a learned per-agent cost critic and
per-(agent, cost) Lagrange multipliers.

  Vh = ValueNet(n_cost, decompose, use_global_info) with its OWN GRU carries (VhGlobalNet), scanned over
       the episode like Vl (scan_Vh, :152-163) plus the final value (:181-190);
  (Qh, Ql) = compute_dec_ocp_gae(max(costs, 0), -reward, Vh, Vl)                           (:193-200)
  A = -norm_t(Ql - Vl) - mean_h(lagr * norm_t(Qh - Vh))                                     (:205-221)
  per minibatch: update_Vl, update_Vh (l2 to Qh, 16-step chunks from zero carries, :246-280),
  update_policy(A), then update_lagr with the UPDATED policy (log pi over whole episodes from zero carries,
  lagr = relu(lagr + lr mean(Vh (1 - gamma) + ratio Ah)), :283-305).
Kernels: the DGPPO networks, dgppo_clip_min0, dgppo_lagr_advantages, dgppo_lagr_update."""
from __future__ import annotations

import warnings

import torch

from ..nn import kernels as K
from ..trainer.rollout import Rollout
from .dgppo import PREPASS_GRAPHS, DGPPO, minibatch_plan
from .informarl import InforMARL
from .module.nets import VhGlobalNet


class InforMARLLagr(InforMARL):
    VH_NET = VhGlobalNet

    def __init__(self, *args, lagr_init: float = 0.78, lr_lagr: float = 1e-7, **kwargs):
        kwargs.pop("cost_weight", None)  # the reference passes 0 to InforMARL (informarl_lagr.py:58-61)
        super().__init__(*args, cost_weight=0.0, **kwargs)
        self.lagr_init, self.lr_lagr = float(lagr_init), float(lr_lagr)
        self.ah_lagr = torch.full((self._n_agents, self._env.n_cost), self.lagr_init, device=self.device)
        self.init_Vh_rnn_state = torch.zeros((self.rnn_layers, self._n_agents, self.n_carries, 64), device=self.device)

    @property
    def config(self) -> dict:
        c = dict(super().config)
        c.update(lr_Vh=self.lr_Vh, Vh_gnn_layers=self.Vh_gnn_layers, lagr_init=self.lagr_init, lr_lagr=self.lr_lagr)
        return c

    def _vh_scan_all(self, rollout: Rollout, chunk: int) -> torch.Tensor:
        """scan_Vh over every env's whole episode from zero carries, plus the final Vh at next_graph[:, -1]
        from the scan's last carries (final_Vh_fn_, informarl_lagr.py:193-203): (B, T+1, n, n_cost)."""
        B, T = rollout.rewards.shape
        n, nh = self._n_agents, self._env.n_cost
        out = torch.empty((B, T + 1, n, nh), device=self.device)
        for e0 in range(0, B, chunk):
            e1 = min(B, e0 + chunk)
            g = self._graphs(rollout.graph, slice(e0, e1))
            v, hT, _ = self.Vh.seq_fwd(g, e1 - e0, T, keep_cache=False)
            out[e0:e1, :T].copy_(v.view(e1 - e0, T, n, nh))
            vf, _, _ = self.Vh.seq_fwd(self._last_graph(rollout.next_graph, slice(e0, e1)), e1 - e0, 1, h0=hT,
                                       keep_cache=False)
            out[e0:e1, T].copy_(vf.view(e1 - e0, n, nh))
        return out

    def update(self, rollout: Rollout, step: int) -> dict:
        env, dev = self._env, self.device
        B, T = rollout.rewards.shape
        n, nh = self._n_agents, env.n_cost
        chunk = max(1, min(B, PREPASS_GRAPHS // T))
        info = {}
        for _ in range(self.epoch_ppo):
            # the Vl and Vh scans are independent: two streams, as DGPPO's prepass
            Vl, Vh = self._parallel([lambda: self._vl_all(rollout, chunk),  # (B, T+1)
                                     lambda: self._vh_scan_all(rollout, chunk)])  # (B, T+1, n, nh)
            hs = torch.empty(rollout.costs.shape, device=dev)  # max(costs, 0) (informarl_lagr.py:197)
            K.clip_min0(rollout.costs.contiguous(), hs)
            Qh = torch.empty((B, T, n, nh), device=dev)
            Ql = torch.empty((B, T), device=dev)
            K.gae(hs, (-rollout.rewards).contiguous(), Vh, Vl, Qh, Ql, self.gamma, self.gae_lambda)
            A = torch.empty((B, T, n), device=dev)
            Ah = torch.empty((B, T, n, nh), device=dev)
            K.lagr_advantages(Ql, Vl, Qh, Vh, self.ah_lagr, A, Ah)
            if self.trace is not None:
                self.trace.update(Vl=Vl.clone(), Vh=Vh.clone(), hs=hs.clone(), Ql=Ql.clone(), Qh=Qh.clone(),
                                  A=A.clone(), Ah=Ah.clone(), lagr0=self.ah_lagr.clone(), mb=[])
            L = self.rnn_step
            assert T % L == 0, "jnp.array(jnp.array_split(...)) in the reference needs rnn_step | T"
            S_per_env = T // L
            Vh_T = Vh[:, :T]
            lagr_mean = torch.empty(1, device=dev)
            batches = minibatch_plan(B, T, self.world, self.batch_size, self.np_rng)
            env_ids = self._env_ids(batches)
            for bi in batches:
                envs = next(env_ids)
                Bm = len(bi)
                self.grad_flat.zero_()
                rg = rollout.graph
                nodes, edges, recv, send, acts, lp_old, adv, tgt, qh, vh_mb, ah_mb = self._gather(
                    envs, rg.nodes, rg.edges, rg.receivers, rg.senders, rollout.actions, rollout.log_pis, A, Ql, Qh,
                    Vh_T, Ah)
                g = self._graph_batch(nodes, edges, recv, send)
                pending = []
                # update_Vl (informarl.py:357-385)
                v, _, cache = self.Vl.seq_fwd(g, Bm * S_per_env, L)
                tgt = tgt.view(Bm * S_per_env, L)
                dv = torch.empty_like(v)
                vl_loss = torch.empty(1, device=dev)
                K.l2_loss(v, tgt, dv, vl_loss)
                self.Vl.seq_bwd(cache, dv)
                del cache
                self._start_reduce(self.Vl, pending)
                # update_Vh (informarl_lagr.py:246-280): 16-step chunks from zero carries, l2 to Qh
                vh, _, cache = self.Vh.seq_fwd(g, Bm * S_per_env, L)
                dvh = torch.empty_like(vh)
                vh_loss = torch.empty(1, device=dev)
                qh = qh.view(-1, nh)
                K.l2_loss(vh, qh, dvh, vh_loss)
                self.Vh.seq_bwd(cache, dvh)
                del cache
                self._start_reduce(self.Vh, pending)
                # update_policy (informarl.py:405-457)
                acts, lp_old, adv = acts.view(-1, self._action_dim), lp_old.view(-1), adv.view(-1)
                lp, ent, cache = self.actor.eval_seq_fwd(g, Bm * S_per_env, L, acts, self.entropy_eps)
                dlp, dent = torch.empty_like(lp), torch.empty_like(ent)
                stats = torch.empty(4, device=dev)
                K.ppo_loss(lp, lp_old, adv, ent, self.clip_eps, self.coef_ent, dlp, dent, stats)
                self.actor.eval_seq_bwd(cache, dlp, dent)
                del cache
                self._start_reduce(self.actor, pending)
                self._finish_reduce(pending)
                if self.trace is not None:
                    self.trace["mb"].append(dict(envs=bi.copy(), grad=self.grad_flat.clone(),
                                                 before={k: o.ps.flat.clone() for k, o in self.opt.items()}))
                for name in ("Vl", "Vh", "policy"):
                    self.opt[name].step()
                # update_lagr with the updated policy: whole episodes from zero carries (informarl_lagr.py:283-305)
                lp_new, _, _ = self.actor.eval_seq_fwd(g, Bm, T, acts, self.entropy_eps)
                if self.world == 1:
                    K.lagr_update(lp_new, lp_old, vh_mb, ah_mb, self.ah_lagr, lagr_mean, Bm * T, self.gamma,
                                  self.lr_lagr)
                else:
                    self._lagr_step_sharded(lp_new, lp_old, vh_mb, ah_mb, Bm * T, lagr_mean)
                if self.trace is not None:
                    self.trace["mb"][-1].update(lp_new=lp_new.clone(), lagr=self.ah_lagr.clone())
                info = {"Vl/loss": vl_loss, "Vl/max_target": tgt.max(), "Vl/min_target": tgt.min(),
                        "Vh/loss": vh_loss, "Vh/max_target": qh.max(), "Vh/min_target": qh.min(),
                        "policy/stats": stats, "policy/log_pi_min": lp_old.min(), "policy/lagr_mean": lagr_mean}
        out = self._finish_info(info)
        out["Vh/grad_norm"] = out.pop("Vh/grad_Vh_norm")
        out["Vh/has_nan"] = out.pop("Vh/grad_Vh_has_nan")
        return out

    def _lagr_step_sharded(self, lp_new, lp_old, vh_mb, ah_mb, rows, lagr_mean):
        """Multi-GPU update_lagr: each rank holds 1/world of the minibatch (equal shards), so the global
        delta is the mean of the per-rank deltas.  The kernel's relu(0 - lr delta) with lr = +1 and -1 gives
        relu(-delta) and relu(delta) of this shard exactly; their difference is the rank's delta, averaged
        over ranks by one all-reduce, then every rank applies relu(lagr - lr_lagr delta) identically."""
        import torch.distributed as dist

        nz, nh = self.ah_lagr.shape
        neg = torch.zeros((nz, nh), device=self.device)
        pos = torch.zeros((nz, nh), device=self.device)
        K.lagr_update(lp_new, lp_old, vh_mb, ah_mb, neg, None, rows, self.gamma, 1.0)  # relu(-delta)
        K.lagr_update(lp_new, lp_old, vh_mb, ah_mb, pos, None, rows, self.gamma, -1.0)  # relu(delta)
        delta = pos - neg
        dist.all_reduce(delta, op=dist.ReduceOp.SUM)
        self.ah_lagr.sub_(delta, alpha=self.lr_lagr / self.world).clamp_(min=0.0)
        torch.mean(self.ah_lagr.view(-1), 0, keepdim=True, out=lagr_mean)

    # checkpoints: params and Adam state as DGPPO (actor / Vl / Vh) plus the multipliers
    def save(self, save_dir: str, step: int):
        import os

        super().save(save_dir, step)
        torch.save({"ah_lagr": self.ah_lagr.cpu()}, os.path.join(save_dir, str(step), "lagr.pt"))

    def load(self, load_dir: str, step: int):
        import os

        super().load(load_dir, step)
        fn = os.path.join(load_dir, str(step), "lagr.pt")
        if os.path.exists(fn):
            lagr = torch.load(fn, weights_only=True)["ah_lagr"]
            # per-(agent, cost) multipliers of the training agent count: an eval on another -n (test.py) does not
            # use them, and the reference's checkpoint holds the networks only (informarl_lagr.py:311-327)
            if lagr.shape == self.ah_lagr.shape:
                self.ah_lagr.copy_(lagr)
                return
            warnings.warn(f"{fn}: multipliers of shape {tuple(lagr.shape)} do not fit this algorithm's "
                          f"{tuple(self.ah_lagr.shape)}; keeping lagr_init (fine for evaluation, not for resuming)")
        else:
            warnings.warn(f"{fn} missing (network-only or reference checkpoint): the Lagrange multipliers keep "
                          "lagr_init (fine for evaluation, not for resuming training)")

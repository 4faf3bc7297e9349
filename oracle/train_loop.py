"""CPU restatement of the whole DGPPO training loop (TEST INFRASTRUCTURE ONLY, see oracle/__init__.py):
Trainer.train (trainer.py:78-141) -> collect (rollout, trainer/utils.py:22-57) -> DGPPO.update
(dgppo.py:136-321 + informarl.py:357-457) with the oracle env (oracle/env.py, NumPy fp32) and the oracle
networks (oracle/nets_t.py, torch autograd on the reference's per-edge formulation).

It shares no code with the GPU product path (no kernels, no ParamSpace layouts, no RolloutEngine), so a
learning curve it produces is the restated reference algorithm's own behaviour: scripts/oracle_learning.py
runs it next to the GPU training to tell "what the algorithm does" from "what the kernels do".
Differences from the GPU run that are not algorithmic: action noise comes from NumPy's default_rng (the
GPU draws Philox), and the networks run in the chosen torch dtype (float32 by default here, for speed).
"""
from __future__ import annotations

import numpy as np
import torch

from . import env as OE
from . import nets as O
from . import nets_t as R

GRAPH_KEYS = ("nodes", "edges", "receivers", "senders")


def _walk_leaves(tree, fn):
    if isinstance(tree, dict):
        return {k: _walk_leaves(v, fn) for k, v in tree.items()}
    if isinstance(tree, list):
        return [_walk_leaves(v, fn) for v in tree]
    return fn(tree)


def _leaves(tree):
    if isinstance(tree, dict):
        for k in tree:
            yield from _leaves(tree[k])
    elif isinstance(tree, list):
        for v in tree:
            yield from _leaves(v)
    else:
        yield tree


def _zip_map(fn, *trees):
    t0 = trees[0]
    if isinstance(t0, dict):
        return {k: _zip_map(fn, *(t[k] for t in trees)) for k in t0}
    if isinstance(t0, list):
        return [_zip_map(fn, *(t[i] for t in trees)) for i in range(len(t0))]
    return fn(*trees)


class AdamTree:
    """optax.apply_if_finite(optax.adam(lr), 1e6) + compute_norm_and_clip (trainer/utils.py:105-118) on a
    flax-layout tree of float64 NumPy leaves."""

    def __init__(self, params, lr, max_norm=2.0):
        self.lr, self.max_norm = lr, max_norm
        self.m = _walk_leaves(params, lambda x: np.zeros_like(x, np.float64))
        self.v = _walk_leaves(params, lambda x: np.zeros_like(x, np.float64))
        self.count = 0

    def step(self, params, grads):
        gl = [np.asarray(g, np.float64) for g in _leaves(grads)]
        if not all(np.isfinite(g).all() for g in gl):
            return params, float("nan")  # apply_if_finite: skip, state unchanged
        norm = float(np.sqrt(sum((g * g).sum() for g in gl)))
        scale = self.max_norm / max(self.max_norm, norm)
        t = self.count + 1
        b1, b2, eps = 0.9, 0.999, 1e-8
        self.m = _zip_map(lambda m, g: b1 * m + (1 - b1) * g * scale, self.m, grads)
        self.v = _zip_map(lambda v, g: b2 * v + (1 - b2) * (g * scale) ** 2, self.v, grads)
        params = _zip_map(lambda p, m, v: p - self.lr * (m / (1 - b1 ** t)) / (np.sqrt(v / (1 - b2 ** t)) + eps),
                          params, self.m, self.v)
        self.count = t
        return params, norm


class OracleDGPPO:
    """DGPPO with the reference defaults (cbf schedule, alpha 10, cbf_eps 1e-2, clip 0.25, coef_ent 1e-2,
    gamma 0.99, lambda 0.95, lr 3e-4 / 1e-3 / 1e-3, max grad norm 2) on the oracle env + networks.
    trees: (actor, Vl, Vh) flax-layout trees (NumPy), e.g. the GPU algorithm's initial `.flax()` trees."""

    def __init__(self, spec, trees, seed=0, batch_size=16384, rnn_step=16, cbf_weight=1.0, cbf_schedule=True,
                 train_steps=200000, coef_ent=1e-2, entropy_eps=None, force_safe=False, dtype=torch.float32):
        self.spec = spec
        self.pa, self.pl, self.ph = (_walk_leaves(t, lambda x: np.asarray(x, np.float64)) for t in trees)
        self.opt = {"policy": AdamTree(self.pa, 3e-4), "Vl": AdamTree(self.pl, 1e-3), "Vh": AdamTree(self.ph, 1e-3)}
        self.batch_size, self.rnn_step = batch_size, rnn_step
        self.cbf_weight, self.cbf_schedule, self.train_steps = cbf_weight, cbf_schedule, int(train_steps)
        self.coef_ent, self.clip_eps, self.gamma, self.lam = coef_ent, 0.25, 0.99, 0.95
        self.alpha, self.cbf_eps, self.force_safe = 10.0, 1e-2, force_safe
        n, A = spec.n, spec.ad
        self.A = A
        self.entropy_eps = (np.random.default_rng(10_000 + seed).standard_normal((n, A)).astype(np.float32)
                            if entropy_eps is None else np.asarray(entropy_eps, np.float32))
        self.np_rng = np.random.default_rng(seed)   # minibatch shuffles (dgppo.py:155-156)
        self.noise_rng = np.random.default_rng(seed + 12345)
        self.dtype = dtype

    def cbf_weight_at(self, step):
        w = self.cbf_weight
        if self.cbf_schedule:
            w *= 2 if step >= int(self.train_steps * 0.5) else 1
            w *= 2 if step >= int(self.train_steps * 0.75) else 1
        return w

    # ---- rollouts (trainer/utils.py:22-86) ----------------------------------------------------------
    def rollout(self, seed, n_env, stochastic=True, T=128):
        spec, n = self.spec, self.spec.n
        agents, goals, third = OE.env_reset(spec, seed, n_env)
        g = OE.initial_graph(spec, agents, goals, third)
        h = np.zeros((n_env, n, 64), np.float32)
        graphs = {k: [] for k in GRAPH_KEYS}
        rnn, acts, lps, rews, costs = [], [], [], [], []
        R.T64 = self.dtype
        try:
            pa = R.to_t(self.pa)
            for t in range(T):
                for k in GRAPH_KEYS:
                    graphs[k].append(g[k])
                with torch.no_grad():
                    h2 = R.actor_carry(pa, g, h, n)
                    mu, sd = R.policy_dist(pa, h2)
                    if stochastic:
                        eps = torch.as_tensor(self.noise_rng.standard_normal(mu.shape), dtype=mu.dtype)
                        a = torch.tanh(mu + sd * eps)
                        lps.append(R.tanh_normal_log_prob(a.numpy().astype(np.float32), mu, sd).numpy())
                    else:
                        a = torch.tanh(mu)
                a = a.numpy().astype(np.float32)
                h2 = h2.numpy().astype(np.float32)
                rnn.append(h if stochastic else h2)  # carry before (rollout) / after (test_rollout) the step
                acts.append(a)
                nxt = OE.env_step(spec, g["states"], third, a)
                rews.append(nxt["reward"])
                costs.append(nxt["cost"])
                g, h = nxt, h2
        finally:
            R.T64 = torch.float64
        st = lambda xs: np.stack(xs, 1)  # noqa: E731  (B, T, ...)
        return dict(graph={k: st(v) for k, v in graphs.items()}, last={k: np.asarray(g[k]) for k in GRAPH_KEYS},
                    rewards=st(rews), costs=st(costs), rnn=st(rnn), actions=st(acts),
                    log_pis=st(lps) if stochastic else None)

    # ---- DGPPO.update (dgppo.py:136-321) ------------------------------------------------------------
    def update(self, roll, det_seed, step):
        spec, n = self.spec, self.spec.n
        B, T = roll["rewards"].shape
        det = self.rollout(det_seed, B, stochastic=False, T=T)
        R.T64 = self.dtype
        try:
            dt, alpha = (np.inf, 0.0) if self.force_safe else (spec.dt, self.alpha)
            pre = R.dgppo_prepass(R.to_t(self.pa), R.to_t(self.pl), R.to_t(self.ph), roll, det, n, dt, self.gamma,
                                  self.lam, alpha, self.cbf_eps, self.cbf_weight_at(step))
            idx = np.arange(B)
            self.np_rng.shuffle(idx)
            batches = np.array_split(idx, B // (self.batch_size // T))
            info = {}
            for envs in batches:
                ts = [R.to_t(x, requires_grad=True) for x in (self.pa, self.pl, self.ph)]
                info = R.dgppo_minibatch_grads(*ts, roll, det, envs, pre["Ql"], pre["Qh_det"], pre["A"], n,
                                               self.rnn_step, self.entropy_eps, self.clip_eps, self.coef_ent)
                ga, gl, gh = (R.grads(t) for t in ts)
                self.pl, info["Vl_grad_norm"] = self.opt["Vl"].step(self.pl, gl)
                self.ph, info["Vh_grad_norm"] = self.opt["Vh"].step(self.ph, gh)
                self.pa, info["policy_grad_norm"] = self.opt["policy"].step(self.pa, ga)
        finally:
            R.T64 = torch.float64
        T_ = T
        d_term = (pre["Vh"][:, 1:] - pre["Vh"][:, :T_]) / spec.dt
        info.update(safe_data=float(pre["safe_data"]), det_cost_mean=[float(x) for x in det["costs"].mean((0, 1, 2))],
                    Vh_mean=[float(x) for x in pre["Vh"].mean((0, 1, 2))],
                    Qh_det_mean=[float(x) for x in pre["Qh_det"].mean((0, 1, 2))],
                    dVh_dt_std=[float(x) for x in d_term.std((0, 1, 2))])
        return info


def eval_metrics(r):
    """trainer.py:103-116 on an oracle rollout dict."""
    rew = r["rewards"].astype(np.float64)
    c = r["costs"].astype(np.float64)
    return {"eval/reward": float(rew.sum(-1).mean()),
            "eval/cost": float(np.maximum(c, 0).max(-1).max(-1).sum(-1).mean()),
            "eval/unsafe_frac": float((c.max(-1).max(-2) >= 1e-6).mean())}


__all__ = ["OracleDGPPO", "AdamTree", "eval_metrics", "O"]

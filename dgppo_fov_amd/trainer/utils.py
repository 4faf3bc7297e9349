"""Evaluation metrics of the reference's Trainer / test.py on (B, T, ...) rollouts.

* `eval_info` = trainer.py:103-116: eval/reward (mean over envs of the episode return),
  eval/reward_final, eval/cost (mean over envs of the sum over t of max over (agent, cost) of
  relu(cost)), eval/unsafe_frac (mean over (env, agent) of [max over (t, cost) of cost >= 1e-6]).
* `safe_rate` = test.py:103-139: per env, 1 - mean over agents of max over t of any(cost >= 0).
Works on torch tensors (device or CPU) or NumPy arrays; returns Python floats."""
from __future__ import annotations

import numpy as np


def _np(x):
    if hasattr(x, "detach"):
        return x.detach().float().cpu().numpy()
    return np.asarray(x)


def eval_info(rewards, costs) -> dict:
    """rewards (B, T), costs (B, T, n, n_cost)."""
    r = _np(rewards).astype(np.float64)
    c = _np(costs).astype(np.float64)
    total = r.sum(axis=-1)
    return {
        "eval/reward": float(total.mean()),
        "eval/reward_final": float(r[:, -1].mean()),
        "eval/cost": float(np.maximum(c, 0.0).max(axis=-1).max(axis=-1).sum(axis=-1).mean()),
        "eval/unsafe_frac": float((c.max(axis=-1).max(axis=-2) >= 1e-6).mean()),
        "eval/reward_min": float(total.min()),
        "eval/reward_max": float(total.max()),
    }


def safe_rate(costs) -> np.ndarray:
    """costs (B, T, n, n_cost) of the pre-step graphs -> per-env safe rate (B,)."""
    c = _np(costs)
    unsafe = (c >= 0.0).any(axis=-1)          # (B, T, n)
    return 1.0 - unsafe.max(axis=1).mean(axis=-1)

"""Why is DGPPO's safe_data so low?  Trace K updates of DGPPO (LidarTarget n=2 obs=0 by default, the
reference defaults otherwise) and print, per update, the statistics of the quantities the safe-set mask
is built from (dgppo.py:218-259): rollout / det-rollout costs, Vh on both rollouts, Qh_det (Vh's
target), the CBF derivative terms (Vh_{t+1} - Vh_t)/dt and alpha Vh_t per cost column, and safe_data.

  python scripts/diag_safe.py [--env LidarTarget -n 2 --obs 0 --updates 40 --rnn-step 128]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgppo_fov_amd.algo import make_algo  # noqa: E402
from dgppo_fov_amd.env import make_env  # noqa: E402


def stats(x):
    x = x.double()
    return [round(float(v), 4) for v in (x.mean(), x.std(), x.min(), x.max())]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--env", default="LidarTarget")
    ap.add_argument("-n", type=int, default=2)
    ap.add_argument("--obs", type=int, default=0)
    ap.add_argument("--updates", type=int, default=40)
    ap.add_argument("--every", type=int, default=5)
    ap.add_argument("--rnn-step", type=int, default=128)
    ap.add_argument("--cbf-weight", type=float, default=1.0)
    ap.add_argument("--n-env", type=int, default=128)
    ap.add_argument("--out", default="gpurun_out/diag_safe.json")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    env = make_env(a.env, a.n, num_obs=a.obs, device=dev)
    algo = make_algo("dgppo", env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                     action_dim=env.action_dim, n_agents=a.n, batch_size=16384, rnn_step=a.rnn_step, seed=0,
                     device=dev, cbf_weight=a.cbf_weight, train_steps=200000)
    rng = np.random.default_rng(0)
    rows = []
    for it in range(a.updates):
        r = algo.collect(algo.params, int(rng.integers(0, 2 ** 62)), n_env=a.n_env)
        rec = it % a.every == 0
        algo.trace = {} if rec else None
        info = algo.update(r, it)
        if not rec:
            continue
        tr = algo.trace
        Vh, Vh_det, Qh_det, Qh = tr["Vh"], tr["Vh_det"], tr["Qh_det"], tr["Qh"]
        T = r.rewards.shape[1]
        d_term = (Vh[:, 1:] - Vh[:, :T]) / env.dt
        a_term = algo.alpha * Vh[:, :T]
        deriv = d_term + a_term
        row = {"update": it, "safe_data": round(info["eval/safe_data"], 4),
               "safe_per_col": [round(float((deriv[..., h] <= 0).float().mean()), 4) for h in range(env.n_cost)],
               "cost_roll": [stats(r.costs[..., h]) for h in range(env.n_cost)],
               "cost_det": [stats(tr["det"].costs[..., h]) for h in range(env.n_cost)],
               "Vh_roll": [stats(Vh[..., h]) for h in range(env.n_cost)],
               "Vh_det": [stats(Vh_det[..., h]) for h in range(env.n_cost)],
               "Qh_roll": [stats(Qh[..., h]) for h in range(env.n_cost)],
               "Qh_det": [stats(Qh_det[..., h]) for h in range(env.n_cost)],
               "dVh_over_dt": [stats(d_term[..., h]) for h in range(env.n_cost)],
               "alpha_Vh": [stats(a_term[..., h]) for h in range(env.n_cost)],
               "Vh_loss": round(info["Vh/loss_Vh"], 5), "act_abs_mean": round(float(r.actions.abs().mean()), 4)}
        rows.append(row)
        print(json.dumps(row), flush=True)
    algo.trace = None
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump({"args": vars(a), "rows": rows, "stats": "[mean, std, min, max]"}, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()

"""The restated reference training loop on the CPU (oracle/train_loop.py: oracle env + autograd networks, no
GPU kernels) from the SAME initial parameters as the GPU DGPPO of the given seed: per update it logs safe_data,
the det-rollout costs, Vh / Qh_det means per cost column and the losses; every --eval-interval updates the
deterministic eval of trainer.py:103-116 on --n-env-test envs.  Compare with scripts/learning_run.py /
scripts/diag_safe.py on the GPU.

  python scripts/oracle_learning.py --env LidarTarget -n 2 --obs 0 --rnn-step 128 --updates 40 --out ...
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgppo_fov_amd.algo.module.nets import ActorNet, VhNet, VlNet  # noqa: E402  (host-side init only)
from oracle import env as OE  # noqa: E402
from oracle.train_loop import OracleDGPPO, eval_metrics  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--env", default="LidarTarget")
    ap.add_argument("-n", type=int, default=2)
    ap.add_argument("--obs", type=int, default=0)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--updates", type=int, default=40)
    ap.add_argument("--rnn-step", type=int, default=128)
    ap.add_argument("--cbf-weight", type=float, default=1.0)
    ap.add_argument("--coef-ent", type=float, default=1e-2)
    ap.add_argument("--force-safe", action="store_true")
    ap.add_argument("--n-env", type=int, default=128)
    ap.add_argument("--n-env-test", type=int, default=32)
    ap.add_argument("--eval-interval", type=int, default=10)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--out", default="gpurun_out/oracle_learning.json")
    a = ap.parse_args()
    if a.threads:
        torch.set_num_threads(a.threads)
    spec = OE.Spec(a.env, a.n, a.obs)
    s = a.seed
    trees = [ActorNet(spec.nd, a.n, "cpu", seed=3 * s, action_dim=spec.ad, edge_dim=spec.ed).flax(),
             VlNet(spec.nd, a.n, "cpu", seed=3 * s + 1, edge_dim=spec.ed).flax(),
             VhNet(spec.nd, a.n, spec.n_cost, "cpu", seed=3 * s + 2, edge_dim=spec.ed).flax()]
    algo = OracleDGPPO(spec, trees, seed=s, rnn_step=a.rnn_step, cbf_weight=a.cbf_weight, coef_ent=a.coef_ent,
                       force_safe=a.force_safe)
    rng = np.random.default_rng(s)
    rows, evals = [], []
    t0 = time.time()
    for it in range(a.updates + 1):
        if it % a.eval_interval == 0:
            ev = eval_metrics(algo.rollout(s, a.n_env_test, stochastic=False))
            evals.append({"step": it, **ev})
            print(json.dumps({"eval": evals[-1]}), flush=True)
        if it == a.updates:
            break
        roll = algo.rollout(int(rng.integers(0, 2 ** 31)), a.n_env, stochastic=True)
        tr = {"train_reward": float(roll["rewards"].sum(-1).mean()),
              "train_unsafe": float((roll["costs"].max(-1).max(-2) >= 1e-6).mean()),
              "act_drift": float(np.abs(roll["actions"].mean((0, 1))).mean())}
        info = algo.update(roll, int(rng.integers(0, 2 ** 31)), it)
        row = {"update": it, **tr, **{k: (round(v, 5) if isinstance(v, float) else [round(x, 4) for x in v])
                                     for k, v in info.items()}, "wall_s": round(time.time() - t0, 1)}
        rows.append(row)
        print(json.dumps(row), flush=True)
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        json.dump({"args": vars(a), "evals": evals, "rows": rows}, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()

"""Diagnostic: does one DGPPO update step move the policy / Vl / Vh losses DOWN on its own minibatch?

Collects a rollout, runs algo.update with a single minibatch (batch_size = B*T) while tracing the
advantages, then re-evaluates the PPO surrogate and the critic losses on the SAME data with the new
parameters.  A sign error anywhere between the losses and Adam shows up as a loss increase."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dgppo_fov_amd.algo import make_algo  # noqa: E402
from dgppo_fov_amd.env import make_env  # noqa: E402
from dgppo_fov_amd.nn import kernels as K  # noqa: E402


def policy_loss(algo, roll, A, envs, L):
    B, T = roll.rewards.shape
    e = torch.as_tensor(envs, device=algo.device)
    g = algo._graphs(roll.graph, e)
    S = len(envs) * (T // L)
    acts = roll.actions.index_select(0, e).reshape(-1, algo.action_dim).contiguous()
    lp_old = roll.log_pis.index_select(0, e).reshape(-1).contiguous()
    adv = A.index_select(0, e).reshape(-1).contiguous()
    lp, ent, _ = algo.actor.eval_seq_fwd(g, S, L, acts, algo.entropy_eps)
    dlp, dent, st = torch.empty_like(lp), torch.empty_like(ent), torch.empty(4, device=algo.device)
    K.ppo_loss(lp, lp_old, adv, ent, algo.clip_eps, algo.coef_ent, dlp, dent, st)
    ratio = torch.exp(lp - lp_old)
    return float(st[0] - algo.coef_ent * st[1]), float((ratio * adv).mean()), float(st[1])


def main():
    dev = torch.device("cuda", 0)
    name = sys.argv[1] if len(sys.argv) > 1 else "dgppo"
    lr = float(sys.argv[2]) if len(sys.argv) > 2 else 3e-4
    env = make_env("LidarSpread", 8, num_obs=3, device=dev)
    B, T, L = 64, env.max_episode_steps, 16
    algo = make_algo(name, env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                     action_dim=env.action_dim, n_agents=8, batch_size=B * T, rnn_step=L, lr_actor=lr,
                     train_steps=200000, seed=0, device=dev)
    for it in range(3):
        roll = algo.collect(algo.params, 100 + it, n_env=B)
        algo.trace = {}
        info = algo.update(roll, it)
        tr = algo.trace
        A = tr["A"]
        (mb,) = tr["mb"]
        envs = mb["envs"]
        # the loss at the pre-update parameters (restore them), then at the updated ones
        after = {k: o.ps.flat.clone() for k, o in algo.opt.items()}
        for k, o in algo.opt.items():
            o.ps.flat.copy_(mb["before"][k])
        l0 = policy_loss(algo, roll, A, envs, L)
        for k, o in algo.opt.items():
            o.ps.flat.copy_(after[k])
        l1 = policy_loss(algo, roll, A, envs, L)
        print(f"iter {it}: policy loss {l0[0]:.5f} -> {l1[0]:.5f} (surrogate mean(ratio*A) {l0[1]:.5f} -> {l1[1]:.5f},"
              f" entropy {l0[2]:.4f} -> {l1[2]:.4f}); info loss {info['policy/loss']:.5f}, A mean {A.mean():.4f} "
              f"std {A.std():.4f}, safe_data {info.get('eval/safe_data', float('nan')):.3f}", flush=True)


if __name__ == "__main__":
    main()

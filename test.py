"""Evaluation of a trained DGPPO checkpoint (test.py of Tw6249/dgppo_fov, the metrics part of
test.py:52-139): episode returns, max cost and safe rate (1 - mean over agents of max over t of
any(cost >= 0)) over --epi episodes of --n-env envs, deterministic (test_rollout) or stochastic."""
import argparse
import os

import numpy as np
import yaml


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--path", type=str, required=True, help="run directory (has config.yaml, models/)")
    ap.add_argument("--step", type=int, default=None, help="checkpoint step (default: latest)")
    ap.add_argument("--epi", type=int, default=5)
    ap.add_argument("--n-env", type=int, default=32)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--stochastic", action="store_true", default=False)
    ap.add_argument("--max-step", type=int, default=None)
    args = ap.parse_args()

    import torch

    from dgppo_fov_amd.algo import make_algo
    from dgppo_fov_amd.env import make_env
    from dgppo_fov_amd.trainer.rollout import RolloutEngine
    from dgppo_fov_amd.trainer.utils import safe_rate

    with open(os.path.join(args.path, "config.yaml")) as f:
        docs = list(yaml.safe_load_all(f))
    cfg = {}
    for d in docs:
        cfg.update(d or {})
    dev = torch.device("cuda", 0)
    env = make_env(cfg["env"], cfg["num_agents"], num_obs=cfg["obs"], n_rays=cfg.get("n_rays", 32),
                   max_step=args.max_step, device=dev)
    algo = make_algo(cfg["algo"], env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                     action_dim=env.action_dim, n_agents=env.num_agents, actor_gnn_layers=cfg["actor_gnn_layers"],
                     Vl_gnn_layers=cfg["Vl_gnn_layers"], Vh_gnn_layers=cfg["Vh_gnn_layers"],
                     batch_size=cfg["batch_size"], rnn_step=cfg["rnn_step"], device=dev)
    model_dir = os.path.join(args.path, "models")
    step = args.step if args.step is not None else max(int(d) for d in os.listdir(model_dir) if d.isdigit())
    algo.load(model_dir, step)
    mode = RolloutEngine.MODE_SAMPLE if args.stochastic else RolloutEngine.MODE_DET
    eng = RolloutEngine(env, args.n_env, env.max_episode_steps, dev, actor=algo.actor, mode=mode)
    rewards, costs, rates = [], [], []
    for i in range(args.epi):
        r = eng.run(args.seed + i)
        epi_reward = r.rewards.sum(1).cpu().numpy()
        epi_cost = r.costs.amax(dim=(1, 2, 3)).cpu().numpy()
        rate = safe_rate(r.costs)
        rewards.append(epi_reward), costs.append(epi_cost), rates.append(rate)
        print(f"epi: {i}, reward: {epi_reward.mean():.3f}, cost: {epi_cost.mean():.3f}, "
              f"safe rate: {rate.mean() * 100:.3f}%")
    rewards, costs, rates = np.concatenate(rewards), np.concatenate(costs), np.concatenate(rates)
    print(f"reward: {rewards.mean():.3f}, min/max reward: {rewards.min():.3f}/{rewards.max():.3f}, "
          f"cost: {costs.mean():.3f}, min/max cost: {costs.min():.3f}/{costs.max():.3f}, "
          f"safe_rate: {rates.mean() * 100:.3f}%")


if __name__ == "__main__":
    main()

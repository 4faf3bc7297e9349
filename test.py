"""Evaluation of a trained checkpoint with the reference's CLI (test.py:22-193 of Tw6249/dgppo_fov):
episode return, max cost and safe rate (1 - mean over agents of max over t of any(cost >= 0),
test.py:100-139), optionally on a different agent / obstacle count or env than training
(-n, --obs, --env), appending `test_log.csv` with --log in the reference's column order
(test.py:142-146).

Episodes are environments: episode i is env i of ONE batched rollout (Philox keyed (--seed, i)),
so `--epi 1000` is a single hipGraph replay over 1000 envs; `--offset k` skips the first k
episodes, as the reference's `test_keys[offset:]` does.  Rendering is out of scope,
so --no-video / --dpi are accepted and ignored; --cpu / --debug too (there is no CPU path)."""
import argparse
import os

import numpy as np
import yaml


def _config(path):
    with open(os.path.join(path, "config.yaml")) as f:
        cfg = {}
        for d in yaml.safe_load_all(f):  # train.py dumps vars(args) then algo.config
            cfg.update(d or {})
    return cfg


def test(args):
    print(f"> Running test.py {args}")
    import torch

    from dgppo_fov_amd.algo import make_algo
    from dgppo_fov_amd.env import make_env
    from dgppo_fov_amd.trainer.rollout import RolloutEngine

    np.random.seed(args.seed)
    cfg = _config(args.path)
    dev = torch.device("cuda", 0)
    num_agents = cfg["num_agents"] if args.num_agents is None else args.num_agents
    env = make_env(env_id=cfg["env"] if args.env is None else args.env, num_agents=num_agents,
                   num_obs=cfg["obs"] if args.obs is None else args.obs, n_rays=cfg.get("n_rays", 32),
                   max_step=args.max_step, full_observation=args.full_observation, device=dev)
    algo = make_algo(cfg["algo"], env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                     action_dim=env.action_dim, n_agents=env.num_agents, cost_weight=cfg.get("cost_weight", 0.0),
                     actor_gnn_layers=cfg["actor_gnn_layers"], Vl_gnn_layers=cfg["Vl_gnn_layers"],
                     Vh_gnn_layers=cfg.get("Vh_gnn_layers", 1), lr_actor=cfg["lr_actor"], lr_Vl=cfg["lr_Vl"],
                     max_grad_norm=2.0, seed=cfg["seed"], use_rnn=cfg.get("use_rnn", True),
                     rnn_layers=cfg.get("rnn_layers", 1), use_lstm=cfg.get("use_lstm", False),
                     batch_size=cfg.get("batch_size", 16384), rnn_step=cfg.get("rnn_step", 16), device=dev)
    model_path = os.path.join(args.path, "models")
    step = args.step if args.step is not None else max(int(d) for d in os.listdir(model_path) if d.isdigit())
    print("step: ", step)
    algo.load(model_path, step)  # the networks are agent-count agnostic: -n may differ from training

    episodes = list(range(args.offset, args.epi))
    if not episodes:
        raise SystemExit(f"--offset {args.offset} leaves no episodes of --epi {args.epi}")
    mode = RolloutEngine.MODE_SAMPLE if args.stochastic else RolloutEngine.MODE_DET
    eng = RolloutEngine(env, len(episodes), env.max_episode_steps, dev, env_offset=args.offset, actor=algo.actor,
                        mode=mode)
    roll = eng.run(args.seed)
    rewards = roll.rewards.sum(1).double().cpu().numpy()  # (epi,)
    costs = roll.costs.amax(dim=(1, 2, 3)).double().cpu().numpy()
    # unsafe_mask on the pre-step graphs: the stored costs ARE env.get_cost(rollout.graph)
    is_unsafe = (roll.costs >= 0.0).any(dim=-1).amax(dim=1).cpu().numpy()  # (epi, n)
    for k, i in enumerate(episodes):
        rate = 1 - is_unsafe[k].mean()
        print(f"epi: {i}, reward: {rewards[k]:.3f}, cost: {costs[k]:.3f}, safe rate: {rate * 100:.3f}%")
    safe_mean, safe_std = (1 - is_unsafe).mean(), (1 - is_unsafe).std()
    print(f"reward: {np.mean(rewards):.3f}, min/max reward: {np.min(rewards):.3f}/{np.max(rewards):.3f}, "
          f"cost: {np.mean(costs):.3f}, min/max cost: {np.min(costs):.3f}/{np.max(costs):.3f}, "
          f"safe_rate: {safe_mean * 100:.3f}%")
    if args.log:
        with open(os.path.join(args.path, "test_log.csv"), "a") as f:
            f.write(f"{env.num_agents},{args.epi},{env.max_episode_steps},{env.area_size},{env.params['n_obs']},"
                    f"{safe_mean * 100:.3f},{safe_std * 100:.3f}\n")
    return dict(reward=float(np.mean(rewards)), cost=float(np.mean(costs)), safe_rate=float(safe_mean))


def main():
    parser = argparse.ArgumentParser()
    parser.add_argument("--path", type=str, required=True)
    parser.add_argument("--no-video", action="store_true", default=False)
    parser.add_argument("--epi", type=int, default=5)
    parser.add_argument("--step", type=int, default=None)
    parser.add_argument("--obs", type=int, default=None)
    parser.add_argument("--stochastic", action="store_true", default=False)
    parser.add_argument("--full-observation", action="store_true", default=False)
    parser.add_argument("--debug", action="store_true", default=False)
    parser.add_argument("--cpu", action="store_true", default=False)
    parser.add_argument("--max-step", type=int, default=None)
    parser.add_argument("--log", action="store_true", default=False)
    parser.add_argument("-n", "--num-agents", type=int, default=None)
    parser.add_argument("--seed", type=int, default=1234)
    parser.add_argument("--env", type=str, default=None)
    parser.add_argument("--offset", type=int, default=0)
    parser.add_argument("--dpi", type=int, default=100)
    test(parser.parse_args())


if __name__ == "__main__":
    main()

"""DGPPO training entry point with the reference's CLI (train.py:15-217 of Tw6249/dgppo_fov) on the
MI355X kernels.  Single GPU: `python train.py --env LidarSpread -n 8 --algo dgppo --obs 3`.
Multi-GPU (env-sharded, RCCL gradient all-reduce): `python -m torch.distributed.run --nnodes=1
--nproc-per-node 8 --master-addr 127.0.0.1 train.py ...` -- `--n-env-train` is per GPU and
`--batch-size` is scaled by the world size (same minibatch count per update)."""
import argparse
import datetime
import json
import os

import numpy as np
import yaml


# flags a resumed run may change; every other flag must match the run it continues (train_args.json)
RESUME_FREE = ("resume", "max_minutes", "log_interval", "gpu", "debug", "log_dir", "name")


def check_resume_args(args, log_dir, world=None):
    """--resume continues a run with ITS hyperparameters: refuse a command line whose flags differ from the ones the
    run started with (saved as train_args.json next to config.yaml), except the resume-only flags.  The world size
    (saved as "_world_size") scales the batch size and the env sharding, so a different one is refused too."""
    path = os.path.join(log_dir, "train_args.json")
    if not os.path.exists(path):
        print(f"> warning: {path} missing (run started before it was written); flags not checked")
        return
    with open(path) as f:
        saved = json.load(f)
    cur = dict(vars(args))
    cur["_world_size"] = int(os.environ.get("WORLD_SIZE", "1")) if world is None else int(world)
    saved.setdefault("_world_size", 1)  # runs saved before the world size was recorded ran on one GPU
    diff = {k: (saved[k], cur.get(k)) for k in saved if k not in RESUME_FREE and saved[k] != cur.get(k)}
    if diff:
        raise SystemExit("--resume: flags differ from the run's own (saved, given): " +
                         ", ".join(f"{k}={v[0]!r} vs {v[1]!r}" for k, v in sorted(diff.items())))


def train(args):
    print(f"> Running train.py {args}")
    if args.resume:
        check_resume_args(args, args.resume.rstrip("/"))
    if args.gpu is not None:
        os.environ["CUDA_VISIBLE_DEVICES"] = str(args.gpu)
        print(f"> Using GPU: {args.gpu}")
    import torch
    import torch.distributed as dist

    from dgppo_fov_amd.algo import make_algo
    from dgppo_fov_amd.env import make_env
    from dgppo_fov_amd.trainer.trainer import Trainer

    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=device)
    rank = dist.get_rank() if world > 1 else 0
    np.random.seed(args.seed)

    env = make_env(env_id=args.env, num_agents=args.num_agents, num_obs=args.obs, n_rays=args.n_rays,
                   full_observation=args.full_observation, device=device)
    env_test = make_env(env_id=args.env, num_agents=args.num_agents, num_obs=args.obs, n_rays=args.n_rays,
                        full_observation=args.full_observation, device=device)
    algo = make_algo(
        algo=args.algo, env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
        action_dim=env.action_dim, n_agents=env.num_agents, cost_weight=args.cost_weight,
        cbf_weight=args.cbf_weight, actor_gnn_layers=args.actor_gnn_layers, Vl_gnn_layers=args.Vl_gnn_layers,
        Vh_gnn_layers=args.Vh_gnn_layers, rnn_layers=args.rnn_layers, lr_actor=args.lr_actor, lr_Vl=args.lr_Vl,
        lr_Vh=args.lr_Vh, max_grad_norm=2.0, alpha=args.alpha, cbf_eps=args.cbf_eps, seed=args.seed,
        batch_size=args.batch_size * world, use_rnn=not args.no_rnn, use_lstm=args.use_lstm,
        coef_ent=args.coef_ent, rnn_step=args.rnn_step, gamma=0.99, clip_eps=args.clip_eps,
        lagr_init=args.lagr_init, lr_lagr=args.lr_lagr, train_steps=args.steps,
        cbf_schedule=not args.no_cbf_schedule, cost_schedule=args.cost_schedule, device=device)
    if args.load_checkpoint:
        print(f"> Loading checkpoint from {args.load_checkpoint}, step {args.load_step}")
        algo.load(args.load_checkpoint, args.load_step)

    if args.resume:
        log_dir = args.resume.rstrip("/")
        run_name = os.path.basename(log_dir)
    else:
        rng_ = np.random.default_rng()
        rand_id = "".join([chr(rng_.integers(65, 91)) for _ in range(4)])
        start_time = int(datetime.datetime.now().strftime("%m%d%H%M%S"))
        base = f"{args.log_dir}/{args.env}/{args.algo}"
        if not args.debug and rank == 0:
            os.makedirs(base, exist_ok=True)
        while os.path.exists(f"{base}/seed{args.seed}_{start_time}_{rand_id}"):
            start_time += 1
        log_dir = f"{base}/seed{args.seed}_{start_time}_{rand_id}"
        run_name = "{}_seed{:03}_{}_{}".format(args.algo, args.seed, start_time, rand_id)
        if args.name is not None:
            run_name = "{}_{}_seed{:03}_{}_{}".format(run_name, args.name, args.seed, start_time, rand_id)
    train_params = {"run_name": run_name, "training_steps": args.steps, "eval_interval": args.eval_interval,
                    "eval_epi": args.eval_epi, "save_interval": args.save_interval,
                    "log_interval": args.log_interval, "max_minutes": args.max_minutes}
    trainer = Trainer(env=env, env_test=env_test, algo=algo, gamma=0.99, log_dir=log_dir,
                      n_env_train=args.n_env_train, n_env_test=args.n_env_test, seed=args.seed,
                      params=train_params, save_log=not args.debug)
    if args.resume:
        st = trainer.load_state(log_dir)
        print(f"> Resuming {log_dir} at step {st['next_step']}")
    elif not args.debug and rank == 0:
        with open(f"{log_dir}/config.yaml", "w") as f:
            yaml.safe_dump(vars(args), f)
            yaml.safe_dump(algo.config, f)
        with open(f"{log_dir}/train_args.json", "w") as f:
            json.dump(dict(vars(args), _world_size=world), f)
    done = trainer.train()
    if world > 1:
        dist.destroy_process_group()
    return done


def main():
    parser = argparse.ArgumentParser()
    parser.add_argument("--env", type=str, required=True)
    parser.add_argument("-n", "--num-agents", type=int, required=True)
    parser.add_argument("--algo", type=str, required=True)
    parser.add_argument("--obs", type=int, required=True)
    parser.add_argument("--seed", type=int, default=0)
    parser.add_argument("--steps", type=int, default=200000)
    parser.add_argument("--name", type=str, default=None)
    parser.add_argument("--debug", action="store_true", default=False)
    parser.add_argument("--gpu", type=int, default=None)
    parser.add_argument("--cost-weight", type=float, default=0.)
    parser.add_argument("--n-rays", type=int, default=32)
    parser.add_argument("--full-observation", action="store_true", default=False)
    parser.add_argument("--clip-eps", type=float, default=0.25)
    parser.add_argument("--lagr-init", type=float, default=0.5)
    parser.add_argument("--lr-lagr", type=float, default=1e-7)
    parser.add_argument("--cbf-weight", type=float, default=1.0)
    parser.add_argument("--cbf-eps", type=float, default=1e-2)
    parser.add_argument("--alpha", type=float, default=10.0)
    parser.add_argument("--no-cbf-schedule", action="store_true", default=False)
    parser.add_argument("--cost-schedule", action="store_true", default=False)
    parser.add_argument("--no-rnn", action="store_true", default=False)
    parser.add_argument("--load-checkpoint", type=str, default=None)
    parser.add_argument("--load-step", type=int, default=None)
    parser.add_argument("--actor-gnn-layers", type=int, default=2)
    parser.add_argument("--Vl-gnn-layers", type=int, default=2)
    parser.add_argument("--Vh-gnn-layers", type=int, default=1)
    parser.add_argument("--lr-actor", type=float, default=3e-4)
    parser.add_argument("--lr-Vl", type=float, default=1e-3)
    parser.add_argument("--lr-Vh", type=float, default=1e-3)
    parser.add_argument("--rnn-layers", type=int, default=1)
    parser.add_argument("--use-lstm", action="store_true", default=False)
    parser.add_argument("--coef-ent", type=float, default=1e-2)
    parser.add_argument("--rnn-step", type=int, default=16)
    parser.add_argument("--n-env-train", type=int, default=128)
    parser.add_argument("--batch-size", type=int, default=16384)
    parser.add_argument("--n-env-test", type=int, default=32)
    parser.add_argument("--log-dir", type=str, default="./logs")
    parser.add_argument("--eval-interval", type=int, default=50)
    parser.add_argument("--eval-epi", type=int, default=1)
    parser.add_argument("--save-interval", type=int, default=50)
    # not reference flags: resumable long runs (trainer_state.json + models/<step>/ with Adam state)
    parser.add_argument("--resume", type=str, default=None, help="continue the run saved in this log dir")
    parser.add_argument("--max-minutes", type=float, default=None, help="save a resumable state and stop after")
    parser.add_argument("--log-interval", type=int, default=1, help="log.jsonl keeps every k-th update")
    args = parser.parse_args()
    if args.load_checkpoint and args.load_step is None:
        parser.error("--load-checkpoint requires --load-step")
    train(args)


if __name__ == "__main__":
    main()

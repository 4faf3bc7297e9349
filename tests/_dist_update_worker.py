"""One rank of tests/test_distributed_gpu.py (started as a subprocess with RANK / WORLD_SIZE /
MASTER_ADDR / MASTER_PORT set): gloo process group, all ranks on cuda:0, DGPPO collect on the rank's
env shard + one traced update; saves the shard's rollouts, the reduced minibatch gradient and the
parameters after Adam to <out>/rank<r>.pt.  Test infrastructure, not a product entry point."""
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from dgppo_fov_amd.algo import make_algo  # noqa: E402
from dgppo_fov_amd.env import make_env  # noqa: E402

ENV, N, OBS, B_LOCAL, T, L = "LidarSpread", 3, 2, 4, 32, 16


def host(r):
    f = lambda G: {k: getattr(G, k).detach().cpu().clone() for k in ("nodes", "edges", "states", "receivers",  # noqa
                                                                     "senders")}
    return dict(graph=f(r.graph), next_graph=f(r.next_graph), actions=r.actions.cpu().clone(),
                rnn_states=r.rnn_states.cpu().clone(), rewards=r.rewards.cpu().clone(), costs=r.costs.cpu().clone(),
                dones=r.dones.cpu().clone(), log_pis=None if r.log_pis is None else r.log_pis.cpu().clone())


def graph_mode(out, knob, backend="gloo"):
    """Two collect + update iterations of 2 minibatches each with the parity trace OFF and DGPPO_UPDATE_GRAPH=knob
    (1: minibatch hipGraph replays with the eager flat all-reduce between them, 0: eager per-net buckets); saves
    the parameters and Adam state of every net.  backend "nccl" (RCCL) at world size 1 forces the collectives
    (DGPPO_FORCE_ALLREDUCE=1) and counts them; backend "none" runs without a process group (the no-reduce path)."""
    os.environ["DGPPO_UPDATE_GRAPH"] = knob
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    calls = []
    if backend != "none":
        if backend == "nccl":
            os.environ["DGPPO_FORCE_ALLREDUCE"] = "1"
            dist.init_process_group("nccl", device_id=dev)
            real = dist.all_reduce

            def counted(t, *a, **k):
                calls.append(int(t.numel()))
                return real(t, *a, **k)

            dist.all_reduce = counted
        else:
            dist.init_process_group("gloo")
    rank = dist.get_rank() if backend != "none" else 0
    world = dist.get_world_size() if backend != "none" else 1
    env = make_env(ENV, N, num_obs=OBS, max_step=T, device=dev)
    algo = make_algo("dgppo", env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                     action_dim=env.action_dim, n_agents=N, batch_size=B_LOCAL * T * world // 2, rnn_step=L,
                     train_steps=100, seed=1, device=dev)
    for it in range(2):
        roll = algo.collect(algo.params, 7 + it, n_env=B_LOCAL)
        algo.update(roll, it)
    torch.cuda.synchronize()
    assert (algo._mbg is not None) == (knob == "1")
    if backend == "nccl":
        assert dist.get_backend() == "nccl" and algo._reduce and calls, calls
        print(f"nccl all_reduce calls: {len(calls)} sizes {sorted(set(calls))}", flush=True)
    tag = "" if backend == "gloo" else backend
    torch.save({k: dict(p=o.ps.flat.cpu().clone(), m=o.m.cpu().clone(), v=o.v.cpu().clone(),
                        state=o.state.cpu().clone()) for k, o in algo.opt.items()},
               os.path.join(out, f"{tag}graph{knob}_rank{rank}.pt"))
    if backend != "none":
        dist.barrier()
        dist.destroy_process_group()


def main(out, algo_name="dgppo"):
    if algo_name.startswith("graph"):
        return graph_mode(out, algo_name[5:])
    for backend in ("nccl", "none"):
        if algo_name.startswith(backend + "graph"):
            return graph_mode(out, algo_name[len(backend) + 5:], backend)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    env = make_env(ENV, N, num_obs=OBS, max_step=T, device=dev)
    extra = dict(lagr_init=0.5, lr_lagr=0.1) if algo_name == "informarl_lagr" else {}
    algo = make_algo(algo_name, env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                     action_dim=env.action_dim, n_agents=N, batch_size=B_LOCAL * T * world, rnn_step=L,
                     train_steps=100, seed=1, device=dev, **extra)
    assert algo.world == world and algo.rank == rank
    roll = algo.collect(algo.params, 7, n_env=B_LOCAL)  # env shard [rank B, (rank + 1) B)
    saved = host(roll)
    algo.trace = {}
    info = algo.update(roll, 3)
    torch.cuda.synchronize()
    (mb,) = algo.trace["mb"]
    torch.save(dict(roll=saved, det=host(algo.trace["det"]) if "det" in algo.trace else None,
                    envs=torch.as_tensor(mb["envs"]),
                    grad=mb["grad"].cpu(), before={k: v.cpu() for k, v in mb["before"].items()},
                    after={k: o.ps.flat.cpu().clone() for k, o in algo.opt.items()},
                    safe=info.get("eval/safe_data"),
                    lagr=algo.ah_lagr.cpu().clone() if hasattr(algo, "ah_lagr") else None),
               os.path.join(out, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1], *sys.argv[2:3])

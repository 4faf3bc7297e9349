"""Multi-rank DGPPO.update on the GPU (dgppo.py:275-289): two ranks (gloo, both on
cuda:0) each update on their own env shard; the all-reduced minibatch gradient equals the
single-process gradient of the same minibatch loss on the union of the two shards (the mean of
the shard gradients = the full-batch gradient, within fp32 summation-order tolerance), and the
parameters after clip + Adam are bit-identical across the ranks."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from dgppo_fov_amd.algo import make_algo
from dgppo_fov_amd.env import make_env
from dgppo_fov_amd.trainer.data import Rollout

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import _dist_update_worker as W  # noqa: E402


def _cat(parts, dev):
    return torch.cat([p.to(dev) for p in parts], 0)


def _run_ranks(tmp_path, mode, world=2):
    port = 29700 + (os.getpid() + 7 * len(mode)) % 200
    procs = []
    for r in range(world):
        envv = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                    MASTER_PORT=str(port))
        envv.pop("DGPPO_UPDATE_GRAPH", None)
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "_dist_update_worker.py"), str(tmp_path),
                                       mode], env=envv, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    for p in procs:
        out, _ = p.communicate(timeout=150)
        assert p.returncode == 0, out.decode()[-3000:]
        print(out.decode()[-400:])


def test_two_rank_minibatch_graphs_match_eager(cuda, tmp_path):
    """the minibatch-hipGraph path with two ranks and the parity trace off (two updates of two
    minibatches: the eager first minibatch, its capture, one replay with the eager all-reduce between the two
    graphs) against the eager per-net-bucket path -- parameters and Adam state bit-identical, and identical across
    the ranks."""
    _run_ranks(tmp_path, "graph1")
    _run_ranks(tmp_path, "graph0")
    ld = lambda k, r: torch.load(os.path.join(tmp_path, f"graph{k}_rank{r}.pt"), weights_only=True)  # noqa: E731
    g1, e1, g1b = ld("1", 0), ld("0", 0), ld("1", 1)
    for net in g1:
        for f in ("p", "m", "v", "state"):
            assert torch.equal(g1[net][f], g1b[net][f]), (net, f, "ranks differ")
            assert torch.equal(g1[net][f], e1[net][f]), (net, f, "graph replay vs eager")
    assert not torch.equal(g1["policy"]["m"], torch.zeros_like(g1["policy"]["m"]))


def test_rccl_world1_reduce_paths_bit_identical(cuda, tmp_path):
    """RCCL executed before any 8-GPU run.  A world-size-1 `nccl` (RCCL) process group with the
    collectives forced on (DGPPO_FORCE_ALLREDUCE=1): the eager path's per-net bucketed async all-reduce + the
    safe-data reduce, and the graph path's flat all-reduce issued eagerly between the two minibatch-graph replays.
    Each is bit-identical to the same run without a process group (no reduce at all)."""
    for mode in ("ncclgraph1", "ncclgraph0", "nonegraph1", "nonegraph0"):
        _run_ranks(tmp_path, mode, world=1)
    ld = lambda f: torch.load(os.path.join(tmp_path, f), weights_only=True)  # noqa: E731
    for knob in ("0", "1"):
        a, b = ld(f"ncclgraph{knob}_rank0.pt"), ld(f"nonegraph{knob}_rank0.pt")
        for net in a:
            for f in ("p", "m", "v", "state"):
                assert torch.equal(a[net][f], b[net][f]), (knob, net, f)
        assert not torch.equal(a["policy"]["m"], torch.zeros_like(a["policy"]["m"]))


@pytest.mark.parametrize("algo_name", ["dgppo", "informarl_lagr"])
def test_two_rank_update_equals_single_process_union(cuda, tmp_path, algo_name):
    """informarl_lagr adds the sharded multiplier step (per-rank delta, one all-reduce, same relu step on
    every rank): multipliers identical across ranks and equal to the single-process union's."""
    world, port = 2, 29700 + os.getpid() % 200
    procs = []
    for r in range(world):
        envv = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                    MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "_dist_update_worker.py"), str(tmp_path),
                                       algo_name],
                                      env=envv, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    for p in procs:
        out, _ = p.communicate(timeout=150)
        assert p.returncode == 0, out.decode()[-3000:]
    res = [torch.load(os.path.join(tmp_path, f"rank{r}.pt"), weights_only=False) for r in range(world)]
    # replicas: identical reduced gradient and bit-identical parameters after Adam
    assert torch.equal(res[0]["grad"], res[1]["grad"])
    for k in res[0]["after"]:
        assert torch.equal(res[0]["after"][k], res[1]["after"][k]), k
    assert res[0]["safe"] == res[1]["safe"]

    # single process on the union of the shards: the same minibatch loss, gradient of the full batch
    env = make_env(W.ENV, W.N, num_obs=W.OBS, max_step=W.T, device=cuda)
    B = W.B_LOCAL * world
    extra = dict(lagr_init=0.5, lr_lagr=0.1) if algo_name == "informarl_lagr" else {}
    algo = make_algo(algo_name, env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                     action_dim=env.action_dim, n_agents=W.N, batch_size=B * W.T, rnn_step=W.L, train_steps=100,
                     seed=1, device=cuda, **extra)
    for k, o in algo.opt.items():  # the ranks' starting parameters (same seed -> same init)
        assert torch.equal(o.ps.flat.cpu(), res[0]["before"][k])

    def rollout(key):
        d = [r[key] for r in res]
        g = lambda f: env._assemble(*[_cat([x[f][k] for x in d], cuda) for k in  # noqa: E731
                                      ("nodes", "edges", "states", "receivers", "senders")], None)
        return Rollout(g("graph"), _cat([x["actions"] for x in d], cuda), _cat([x["rnn_states"] for x in d], cuda),
                       _cat([x["rewards"] for x in d], cuda), _cat([x["costs"] for x in d], cuda),
                       _cat([x["dones"] for x in d], cuda),
                       None if d[0]["log_pis"] is None else _cat([x["log_pis"] for x in d], cuda), g("next_graph"))

    roll = rollout("roll")
    if res[0]["det"] is not None:
        det = rollout("det")
        algo.det_rollout = lambda n_env, key: det  # the ranks' deterministic rollouts, concatenated
    algo.trace = {}
    info = algo.update(roll, 3)
    torch.cuda.synchronize()
    (mb,) = algo.trace["mb"]
    assert sorted(mb["envs"].tolist()) == list(range(B))
    g1, g2 = mb["grad"].cpu().double().numpy(), res[0]["grad"].double().numpy()
    off = 0
    for name, net in (("Vl", algo.Vl), ("Vh", algo.Vh), ("policy", algo.actor)):
        a, b = g2[off:off + net.ps.size], g1[off:off + net.ps.size]
        off += net.ps.size
        err = np.abs(a - b).max()
        assert err <= 1e-5 * np.abs(b).max() + 1e-7, f"{name}: shard-mean vs full-batch gradient {err:.3e}"
    if algo_name == "dgppo":
        assert abs(info["eval/safe_data"] - res[0]["safe"]) < 1e-6
    else:
        assert torch.equal(res[0]["lagr"], res[1]["lagr"])
        lg = algo.ah_lagr.cpu()
        assert not torch.equal(lg, torch.full_like(lg, 0.5))  # the step moved the multipliers
        assert (lg - res[0]["lagr"]).abs().max().item() <= 1e-5 * lg.abs().max().item() + 1e-7

"""Multi-GPU logic of the DGPPO update on CPU (gloo, world size 2): the sharded
minibatch plan and the one-collective gradient mean used by DGPPO.update, run through the same
functions the GPU path calls (dgppo_fov_amd/algo/dgppo.py)."""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from dgppo_fov_amd.algo.dgppo import allreduce_mean_, minibatch_plan


def test_minibatch_plan_single_rank_matches_reference_split():
    rng = np.random.default_rng(0)
    plan = minibatch_plan(4096, 128, 1, 16384, rng)
    assert len(plan) == 32 and all(len(b) == 128 for b in plan)
    assert np.array_equal(np.sort(np.concatenate(plan)), np.arange(4096))
    # same shuffle + split as the reference's np.random.shuffle / jnp.array_split
    idx = np.arange(4096)
    np.random.default_rng(0).shuffle(idx)
    assert all(np.array_equal(a, b) for a, b in zip(plan, np.array_split(idx, 32)))
    # batch_size that does not divide B but splits it evenly (reference: 100 envs, 24-env target)
    assert [len(b) for b in minibatch_plan(100, 1, 1, 24, rng)] == [25, 25, 25, 25]
    with pytest.raises(ValueError):
        minibatch_plan(100, 1, 1, 30, rng)  # 3 minibatches of 34/33/33: unequal, as the reference


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        B_local, T, bs = 64, 16, 256  # global minibatch = 16 envs -> 8 per rank, 8 minibatches
        plan = minibatch_plan(B_local, T, world, bs, np.random.default_rng(100 + rank))
        g = torch.arange(10, dtype=torch.float32) * (rank + 1)
        allreduce_mean_(g, world)
        safe = torch.tensor([float(rank + 1)])
        dist.all_reduce(safe)
        out[rank] = (len(plan), [len(b) for b in plan], g.tolist(), float(safe.item()),
                     sorted(np.concatenate(plan).tolist()))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_gradient_mean_and_shards():
    world = 2
    port = 29500 + os.getpid() % 1000
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
        res = dict(out)
    for r in range(world):
        n_mb, sizes, g, safe, envs = res[r]
        assert n_mb == 8 and sizes == [8] * 8          # 8 local + 8 remote envs = 16 per minibatch
        assert envs == list(range(64))                 # every local env exactly once per epoch
        assert np.allclose(g, np.arange(10) * 1.5)     # mean of rank grads (x1, x2)
        assert safe == 3.0
    assert res[0][2] == res[1][2]                      # replicas get identical gradients

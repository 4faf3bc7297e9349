"""The graph-form MFMA attention kernels (csrc/attn_gm.h: a wave per graph, logits / weighted sums / sender
gradients as fp32 MFMA tile products) against the row-block and graph kernels they replace
(dgppo_gnn_set_attn_kernel(0)), through the networks on minibatch-sized graph batches of every env family they
cover (N <= 96 nodes, n <= 10 agents): actor log pi / entropy, Vl and Vh outputs and every parameter gradient.
Both are fp32 with different summation orders, so outputs agree to 1e-5 relative and gradients to 1e-4 of each
tensor's scale (ReLU gates that fp32 rounding decides may differ; the float64 oracle tests in test_nets_gpu.py
pin each kernel family on its own)."""
import numpy as np
import pytest
import torch

from dgppo_fov_amd import _lib
from dgppo_fov_amd.algo.module.nets import ActorNet, VhNet, VlNet

from test_nets_gpu import _graphs, _walk

pytestmark = pytest.mark.gpu

ENVS = [("LidarSpread", 8, 3), ("LidarTarget", 8, 3), ("LidarBicycleTarget", 8, 3), ("MPESpread", 3, 3),
        ("MPETarget", 3, 0), ("LidarOmniTarget", 8, 3), ("LidarLine", 6, 3), ("VMASWheel", 3, 0)]


def _mode(m):
    return _lib.load().dgppo_gnn_set_attn_kernel(m)


def _net_run(net_kind, env, gb, S, L, n, cuda):
    torch.manual_seed(0)
    rng = np.random.default_rng(1)
    if net_kind == "actor":
        net = ActorNet(env.node_dim, n, cuda, seed=3, action_dim=env.action_dim, edge_dim=env.edge_dim)
        acts = torch.from_numpy(rng.uniform(-0.99, 0.99, (S * L * n, env.action_dim)).astype(np.float32)).to(cuda)
        eps = torch.from_numpy(rng.standard_normal((n, env.action_dim)).astype(np.float32)).to(cuda)
        lp, ent, cache = net.eval_seq_fwd(gb, S, L, acts, eps)
        w1 = torch.from_numpy(rng.standard_normal(lp.shape).astype(np.float32)).to(cuda)
        w2 = torch.from_numpy(rng.standard_normal(ent.shape).astype(np.float32)).to(cuda)
        outs = [lp.clone(), ent.clone()]
        net.ps.zero_grad()
        net.eval_seq_bwd(cache, w1, w2)
    elif net_kind == "Vl":
        net = VlNet(env.node_dim, n, cuda, seed=5, edge_dim=env.edge_dim)
        v, _, cache = net.seq_fwd(gb, S, L)
        outs = [v.clone()]
        net.ps.zero_grad()
        net.seq_bwd(cache, torch.from_numpy(rng.standard_normal(v.shape).astype(np.float32)).to(cuda))
    else:
        net = VhNet(env.node_dim, n, env.n_cost, cuda, seed=7, edge_dim=env.edge_dim)
        h = torch.from_numpy(rng.standard_normal((S * L * n, net.carry_width)).astype(np.float32) * 0.5).to(cuda)
        out, cache = net.fwd(gb, h)
        outs = [out.clone()]
        net.ps.zero_grad()
        net.bwd(cache, torch.from_numpy(rng.standard_normal(out.shape).astype(np.float32)).to(cuda))
    torch.cuda.synchronize()
    net.ps.swap_views()
    g = net.flax()
    net.ps.swap_views()
    return [o.cpu().numpy() for o in outs], g


@pytest.mark.parametrize("net_kind", ["actor", "Vl", "Vh"])
@pytest.mark.parametrize("eid,n,obs", ENVS)
def test_gm_matches_rowblock_kernels(cuda, eid, n, obs, net_kind):
    S, L = 24, 16  # 384 graphs (more than one graph per wave of the persistent grid on the small configs)
    env, gb, _ = _graphs(cuda, eid, n, obs, S, L, seed=11)
    prev = _mode(1)
    try:
        res = {}
        for m in (1, 0):
            _mode(m)
            res[m] = _net_run(net_kind, env, gb, S, L, n, cuda)
    finally:
        _mode(max(prev, 0))
    (o1, g1), (o0, g0) = res[1], res[0]
    for a, b in zip(o1, o0):
        err = np.abs(a - b) - (1e-5 + 1e-5 * np.abs(b))
        assert err.max() <= 0, f"{net_kind} output: max abs err {np.abs(a - b).max():.3e}"
    for path, a, b in _walk(g1, g0):
        a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
        scale = np.abs(b).max()
        assert np.abs(a - b).max() <= 1e-4 * scale + 1e-7, f"{net_kind} grad {path}: {np.abs(a - b).max():.3e} vs {scale:.3e}"


def test_gm_selector_roundtrip():
    lib = _lib.load()
    prev = lib.dgppo_gnn_set_attn_kernel(0)
    assert lib.dgppo_gnn_set_attn_kernel(1) == 0
    assert lib.dgppo_gnn_set_attn_kernel(2) == -22
    lib.dgppo_gnn_set_attn_kernel(max(prev, 0))

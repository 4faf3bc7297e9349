"""The fused GraphTransformer layer forward (dgppo_gnn_layer_fwd, ABI 11) against the unfused chain it replaces
([qt | beta] GEMM + dgppo_gnn_attn_fwd + message / update GEMMs, nn/layers.py with DGPPO_FUSED_LAYER off), layer
by layer on env graphs: Y, [qt | beta], attn and xcat agree to fp32 rounding (the two use different summation
orders: |a - b| <= 2e-6 + 2e-5 |b|), the never-receivers' ReLU gates exactly (their rows are computed in the
row-block kernels' order), forward-only calls write Y alone, and the dispatch falls back where the kernel does not
apply.  The networks' forward and gradients against the float64 oracle run through the fused path in
tests/test_nets_gpu.py (it is the default)."""
import numpy as np
import pytest
import torch

from dgppo_fov_amd.algo.module.nets import ActorNet, VhNet
from dgppo_fov_amd.nn import layers
from dgppo_fov_amd.nn.layers import GraphBatch
from dgppo_fov_amd.env import make_env

pytestmark = pytest.mark.gpu


def _batch(cuda, eid, n, obs, S=24, L=3, seed=0):
    env = make_env(eid, n, num_obs=obs, device=cuda)
    g = env.reset(key=seed, n_env=S)
    gs = []
    rng = np.random.default_rng(seed)
    for _ in range(L):
        gs.append(g)
        a = torch.from_numpy(rng.uniform(-1, 1, (S, n, env.action_dim)).astype(np.float32)).to(cuda)
        g = env.step(g, a).graph
    st = lambda f: torch.stack([getattr(x, f) for x in gs], 1).contiguous()  # noqa: E731
    nodes, edges, recv, send = st("nodes"), st("edges"), st("receivers"), st("senders")
    gb = GraphBatch(nodes.view(S * L, *nodes.shape[2:]), edges.view(S * L, *edges.shape[2:]), recv.view(S * L, -1),
                    send.view(S * L, -1), n, env.agent_candidates(cuda), raw_cols=env.nonagent_feature_cols)
    return env, gb.prepare()


def _close(a, b, what, rtol=2e-5, atol=2e-6):
    a, b = a.double().cpu(), b.double().cpu()
    err = ((a - b).abs() - (atol + rtol * b.abs())).max().item()
    assert err <= 0, f"{what}: max abs err {(a - b).abs().max().item():.3e}"


def _run(gnn, g, fused, keep=True):
    old = layers.FUSED_LAYER
    layers.FUSED_LAYER = fused
    try:
        outs, Y = [], None
        for i, L in enumerate(gnn.layers[:2]):
            Y, c = L.fwd(g, keep=keep) if i == 0 else L.fwd(g, xa=Y, pre=gnn.layers[0], keep=keep)
            assert L.last_fused == fused, f"layer {i}: fused path {'not ' if fused else ''}taken"
            outs.append((Y.clone(), c))
        return outs
    finally:
        layers.FUSED_LAYER = old


@pytest.mark.parametrize("eid,n,obs", [("LidarSpread", 8, 3), ("LidarSpread", 3, 2), ("MPESpread", 3, 3),
                                       ("LidarBicycleTarget", 8, 3), ("MPETarget", 3, 0), ("LidarSpread", 5, 1)])
def test_fused_layer_matches_unfused_chain(cuda, eid, n, obs):
    env, g = _batch(cuda, eid, n, obs)
    actor = ActorNet(env.node_dim, n, cuda, seed=3, edge_dim=env.edge_dim)
    vh = VhNet(env.node_dim, n, env.n_cost, cuda, seed=4, edge_dim=env.edge_dim)
    for net in (actor, vh):
        f, u = _run(net.gnn, g, True), _run(net.gnn, g, False)
        for li, ((Yf, cf), (Yu, cu)) in enumerate(zip(f, u)):
            _close(Yf, Yu, f"{eid} layer {li} Y")
            _close(cf[3], cu[3], f"{eid} layer {li} [qt | beta]")
            _close(cf[4], cu[4], f"{eid} layer {li} attn")
            _close(cf[5], cu[5], f"{eid} layer {li} xcat")
            # ReLU gates of the outputs agree except where the unfused pre-activation is within rounding of zero
            assert ((Yf > 0) != (Yu > 0)).sum().item() <= max(2, Yf.numel() // 20000)
    # forward only: Y alone, identical to the cached call's Y (same kernel, fewer stores)
    for (Yk, _), (Yn, cn) in zip(_run(actor.gnn, g, True), _run(actor.gnn, g, True, keep=False)):
        assert cn is None and torch.equal(Yk, Yn)


@pytest.mark.parametrize("eid,n,obs", [("LidarOmniTarget", 3, 2), ("LidarSpread", 32, 8), ("VMASWheel", 3, 0)])
def test_fused_layer_falls_back_outside_its_scope(cuda, eid, n, obs):
    """10-wide edges (Wex), 72 candidates per agent, 13-wide raw rows: the unfused chain runs."""
    env, g = _batch(cuda, eid, n, obs, S=2, L=2)
    actor = ActorNet(env.node_dim, n, cuda, seed=3, edge_dim=env.edge_dim, action_dim=env.action_dim)
    Y, c = actor.gnn.layers[0].fwd(g)
    assert not actor.gnn.layers[0].last_fused and c is not None

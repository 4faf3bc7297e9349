"""Host-side layer logic that needs no GPU: the flax <-> kernel parameter layout of GraphTransformer for
4- and 10-wide edges (Dense_3 split into Wcat's edge rows + Wex), and GraphBatch's wide-node views."""
import numpy as np
import pytest
import torch

from dgppo_fov_amd.nn.layers import GraphBatch, GraphTransformer, ParamSpace


@pytest.mark.parametrize("ED", [4, 10])
def test_graph_transformer_flax_roundtrip(ED):
    ps = ParamSpace()
    L = GraphTransformer(ps, "t", 10, 32, 3, ED)
    ps.build("cpu")
    L.init_host(np.random.default_rng(0))
    d = L.flax()
    rng = np.random.default_rng(1)
    for k in ("Dense_0", "Dense_1", "Dense_2", "Dense_3", "Dense_4"):
        for kk in d[k]:
            d[k][kk] = rng.standard_normal(d[k][kk].shape).astype(np.float32)
    assert d["Dense_3"]["kernel"].shape == (ED, 96)
    L.load_flax(d)
    back = L.flax()
    for k in d:
        for kk in d[k]:
            assert np.array_equal(back[k][kk], d[k][kk]), (k, kk)
    if ED > 4:  # Wex row h*EX + j = Dense_3 row 4 + j, head h's column block
        wex = L.v("Wex").numpy()
        assert np.array_equal(wex[1 * (ED - 4) + 2], d["Dense_3"]["kernel"][4 + 2, 32:64])


def test_omni_graph_batch_views():
    """LidarOmniTarget graphs (oracle reset): never-receiving nodes are zero outside
    nonagent_feature_cols, so the agent-mode layers' compressed raw rows lose nothing; edge views split
    at column 4; nodes wider than 8 without raw_cols are refused."""
    from dgppo_fov_amd.env.lidar_env.lidar_omni_target import LidarOmniTarget
    from oracle import env as OE

    cols = LidarOmniTarget.nonagent_feature_cols
    n = 3
    spec = OE.Spec("LidarOmniTarget", n, 2)
    ag, gl, third = OE.env_reset(spec, 5, 4)
    g = OE.initial_graph(spec, ag, gl, third)
    nodes, edges = g["nodes"], g["edges"]
    mask = np.ones(nodes.shape[2], bool)
    mask[list(cols)] = False
    assert np.abs(nodes[:, n:][..., mask]).max() == 0
    assert np.abs(nodes[:, n:][..., list(cols)]).max() > 0
    G = nodes.shape[0]
    cand = torch.zeros((n, 4), dtype=torch.int32)
    args = (torch.from_numpy(nodes), torch.from_numpy(edges), torch.from_numpy(g["receivers"]),
            torch.from_numpy(g["senders"]), n, cand)
    gb = GraphBatch(*args, raw_cols=cols)
    raw, c = gb.sender_raw
    assert raw.shape == (G, nodes.shape[1], len(cols)) and raw.is_contiguous()
    assert torch.equal(raw, torch.from_numpy(nodes[..., list(cols)].copy()))
    assert torch.equal(gb.edges_head, torch.from_numpy(edges[..., :4].copy()))
    assert torch.equal(gb.edges_x, torch.from_numpy(edges[..., 4:].copy()))
    with pytest.raises(NotImplementedError):
        GraphBatch(*args).sender_raw

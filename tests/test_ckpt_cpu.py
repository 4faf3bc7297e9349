"""Checkpoint interop on the host: reference-layout flax trees (flattened to
.npz with '/'-joined paths) load into the nets and round-trip exactly, with the
autonamed submodules (PolicyNet_*, RNN_*, GRUCell_*) located by their keys.  Parity unpinned against
real reference checkpoints: none ship with the reference, and this package does not unpickle."""
import types

import numpy as np
import pytest

from dgppo_fov_amd.algo.module.nets import ActorNet, VhNet, VlNet
from dgppo_fov_amd.utils import flax_ckpt as FC


def _nets(seed, edge_dim=4, node_dim=7, A=2, n_cost=2, **rk):
    return types.SimpleNamespace(
        actor=ActorNet(node_dim, 3, "cpu", seed=seed, action_dim=A, edge_dim=edge_dim, **rk),
        Vl=VlNet(node_dim, 3, "cpu", seed=seed + 1, edge_dim=edge_dim, **rk),
        Vh=VhNet(node_dim, 3, n_cost, "cpu", seed=seed + 2, edge_dim=edge_dim, **rk))


@pytest.mark.parametrize("edge_dim,node_dim,A,n_cost", [(4, 7, 2, 2), (10, 10, 3, 5)])
def test_reference_npz_round_trip(tmp_path, edge_dim, node_dim, A, n_cost):
    a = _nets(1, edge_dim, node_dim, A, n_cost)
    b = _nets(7, edge_dim, node_dim, A, n_cost)
    FC.save_reference_npz(a, str(tmp_path))
    FC.load_reference_npz(b, str(tmp_path))
    for k in ("actor", "Vl", "Vh"):
        assert np.array_equal(getattr(a, k).ps.flat.numpy(), getattr(b, k).ps.flat.numpy()), k


@pytest.mark.parametrize("rnn,layers", [("gru", 2), ("lstm", 1), ("lstm", 3), ("none", 1)])
def test_reference_npz_round_trip_rnn_options(tmp_path, rnn, layers):
    """--rnn-layers / --use-lstm / --no-rnn: the cells sit under RNN_0 as GRUCell_k / LSTMCell_k (ii..ho)."""
    a = _nets(1, rnn=rnn, rnn_layers=layers)
    b = _nets(5, rnn=rnn, rnn_layers=layers)
    FC.save_reference_npz(a, str(tmp_path))
    flat = FC.flatten(FC.actor_reference_tree(a.actor))
    cell = "LSTMCell" if rnn == "lstm" else "GRUCell"
    names = {k.split("/")[3] for k in flat if "/RNN_0/" in k}
    assert names == ({f"{cell}_{k}" for k in range(layers)} if rnn != "none" else set())
    if rnn == "lstm":
        assert flat["params/PolicyNet_0/RNN_0/LSTMCell_0/hf/bias"].shape == (64,)
        assert "params/PolicyNet_0/RNN_0/LSTMCell_0/if/bias" not in flat
    FC.load_reference_npz(b, str(tmp_path))
    for k in ("actor", "Vl", "Vh"):
        assert np.array_equal(getattr(a, k).ps.flat.numpy(), getattr(b, k).ps.flat.numpy()), k


def test_reference_tree_paths_and_autonames(tmp_path):
    a = _nets(2)
    tree = FC.actor_reference_tree(a.actor)
    flat = FC.flatten(tree)
    assert "params/PolicyNet_0/GraphTransformerGNN_0/GraphTransformer_1/Dense_3/kernel" in flat
    assert "params/PolicyNet_0/PolicyGNNHead/LayerNorm_1/scale" in flat
    assert "params/OutputDenseStdTrans/bias" in flat
    assert flat["params/PolicyNet_0/GraphTransformerGNN_0/GraphTransformer_0/Dense_3/kernel"].shape == (4, 96)
    # other autoname suffixes (e.g. GRUCell_1 when RNN constructs a probe cell first) load the same
    renamed = {k.replace("PolicyNet_0", "PolicyNet_2").replace("GRUCell_0", "GRUCell_1").replace("RNN_0", "RNN_5"): v
               for k, v in flat.items()}
    b = _nets(9)
    b.actor.load_flax(FC.actor_tree(FC.unflatten(renamed)))
    assert np.array_equal(a.actor.ps.flat.numpy(), b.actor.ps.flat.numpy())
    # a tree with two GRU cells is ambiguous and refused
    bad = FC.unflatten(flat)
    bad["params"]["extra"] = {"GRUCell_0": bad["params"]["PolicyNet_0"]["RNN_0"]["GRUCell_0"]}
    with pytest.raises(ValueError):
        FC.actor_tree(bad)

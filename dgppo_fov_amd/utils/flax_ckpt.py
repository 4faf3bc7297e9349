"""Checkpoint interop with the reference's flax parameter trees.

The reference saves `models/<step>/{actor,Vl,Vh}.pkl` = pickled flax param dicts
(`algo/informarl_lagr.py:311-317`).  This package never unpickles anything.  The interchange format is
an `.npz` of plain float32 arrays keyed by the '/'-joined flax paths, which the reference side writes
from its in-memory params next to its own pickle dump (INTEGRATION.md shows the two-line addition to
`save()`); this module reads those files with `numpy.load(allow_pickle=False)` and maps them onto the
kernels' layouts.

Tree shapes (flax autonaming; the submodule names that carry an index suffix are located by the keys
they hold, so the exact suffixes do not matter):
  actor (TanhNormal, `algo/module/policy.py:46-73`):
      PolicyNet_* / GraphTransformerGNN_* / GraphTransformer_{0,1} / Dense_{0..4}   (`nn/gnn.py:78-142`)
      PolicyNet_* / PolicyGNNHead / {Dense_0, LayerNorm_0, Dense_1, LayerNorm_1}     (`nn/mlp.py:6-30`)
      PolicyNet_* / RNN_* / GRUCell_* / {ir, iz, in, hr, hz, hn}                     (`nn/rnn.py:10-30`)
      ScaleHid, OutputDenseMean, OutputDenseStdTrans
  Vl / Vh (RStateFn / DecRStateFn, `algo/module/value.py:15-79`):
      GraphTransformerGNN_* / ..., ValueGNNHead / ..., RNN_* / GRUCell_* / ..., Dense_0 (the output)
"""
from __future__ import annotations

import os

import numpy as np

GRU_KEYS = {"ir", "iz", "in", "hr", "hz", "hn"}
LSTM_KEYS = {"ii", "if", "ig", "io", "hi", "hf", "hg", "ho"}
HEAD_KEYS = {"Dense_0", "LayerNorm_0", "Dense_1", "LayerNorm_1"}


def flatten(tree, prefix="") -> dict:
    out = {}
    for k, v in tree.items():
        p = f"{prefix}/{k}" if prefix else str(k)
        if isinstance(v, dict):
            out.update(flatten(v, p))
        else:
            out[p] = np.asarray(v, np.float32)
    return out


def unflatten(flat: dict) -> dict:
    tree: dict = {}
    for path, v in flat.items():
        d = tree
        parts = path.split("/")
        for p in parts[:-1]:
            d = d.setdefault(p, {})
        d[parts[-1]] = v
    return tree


def _subtrees(tree, path=()):
    yield path, tree
    for k, v in tree.items():
        if isinstance(v, dict):
            yield from _subtrees(v, path + (k,))


def _find(tree, pred, what):
    hits = [(p, t) for p, t in _subtrees(tree) if pred(p, t)]
    if len(hits) != 1:
        raise ValueError(f"reference tree: expected one {what}, found {len(hits)} ({[('/'.join(p)) for p, _ in hits]})")
    return hits[0]


def _strip_params(tree):
    return tree["params"] if set(tree) == {"params"} else tree


def _gnn_layers(tree):
    _, g = _find(tree, lambda p, t: "GraphTransformer_0" in t, "GraphTransformerGNN")
    n = sum(1 for k in g if k.startswith("GraphTransformer_"))
    return [g[f"GraphTransformer_{i}"] for i in range(n)], g


def _gru(tree):
    """The RNN cells (nn/rnn.py:10-30) in the layout RNNStack.load_flax takes: one GRUCell tree (the 1-layer GRU
    default), else the list of GRUCell / LSTMCell trees ordered by their autoname index ([] without an RNN)."""
    cells = [(p, t) for p, t in _subtrees(tree) if GRU_KEYS <= set(t) or LSTM_KEYS <= set(t)]
    if len({p[:-1] for p, _ in cells}) > 1:
        raise ValueError(f"reference tree: RNN cells under more than one parent ({['/'.join(p) for p, _ in cells]})")
    cells.sort(key=lambda pt: int(pt[0][-1].rsplit("_", 1)[-1]) if pt[0] and pt[0][-1].rsplit("_", 1)[-1].isdigit()
               else 0)
    if len(cells) == 1 and GRU_KEYS <= set(cells[0][1]):
        return cells[0][1]
    return [t for _, t in cells]


def _rnn_ref(d):
    """RNNStack.flax() -> the reference's RNN_0 subtree (cells under their autonames), or {} without an RNN."""
    cells = [d] if isinstance(d, dict) else d
    return {"RNN_0": {f"{'LSTMCell' if 'ii' in c else 'GRUCell'}_{k}": c for k, c in enumerate(cells)}} if cells else {}


def _head(tree, name):
    return _find(tree, lambda p, t: bool(p) and p[-1] == name and HEAD_KEYS <= set(t), name)[1]


def actor_tree(ref) -> dict:
    """reference actor params -> ActorNet.load_flax layout"""
    ref = _strip_params(ref)
    layers, _ = _gnn_layers(ref)
    return {"gnn": layers, "head": _head(ref, "PolicyGNNHead"), "gru": _gru(ref), "ScaleHid": ref["ScaleHid"],
            "OutputDenseMean": ref["OutputDenseMean"], "OutputDenseStdTrans": ref["OutputDenseStdTrans"]}


def value_tree(ref) -> dict:
    """reference Vl / Vh params -> VlNet / VhNet.load_flax layout (output Dense = the root's Dense_0)"""
    ref = _strip_params(ref)
    layers, _ = _gnn_layers(ref)
    return {"gnn": layers, "head": _head(ref, "ValueGNNHead"), "gru": _gru(ref), "out": ref["Dense_0"]}


def actor_reference_tree(net) -> dict:
    """ActorNet -> the reference's actor tree (inverse of actor_tree; GRU under the autonames RNN_0/GRUCell_0)."""
    d = net.flax()
    base = {"GraphTransformerGNN_0": {f"GraphTransformer_{i}": L for i, L in enumerate(d["gnn"])},
            "PolicyGNNHead": d["head"], **_rnn_ref(d["gru"])}
    return {"params": {"PolicyNet_0": base, "ScaleHid": d["ScaleHid"], "OutputDenseMean": d["OutputDenseMean"],
                       "OutputDenseStdTrans": d["OutputDenseStdTrans"]}}


def value_reference_tree(net) -> dict:
    d = net.flax()
    return {"params": {"GraphTransformerGNN_0": {f"GraphTransformer_{i}": L for i, L in enumerate(d["gnn"])},
                       "ValueGNNHead": d["head"], **_rnn_ref(d["gru"]), "Dense_0": d["out"]}}


def load_reference_npz(algo, model_dir: str) -> None:
    """Load reference-layout `{actor,Vl,Vh}.npz` into a DGPPO instance's nets.
    Optimizer state is not part of the reference checkpoint and is left untouched."""
    for name, net, conv in (("actor", algo.actor, actor_tree), ("Vl", algo.Vl, value_tree), ("Vh", algo.Vh, value_tree)):
        with np.load(os.path.join(model_dir, f"{name}.npz"), allow_pickle=False) as z:
            ref = unflatten({k: z[k] for k in z.files})
        net.load_flax(conv(ref))


def save_reference_npz(algo, model_dir: str) -> None:
    """Write the nets as reference-layout `{actor,Vl,Vh}.npz` (flattened flax trees)."""
    os.makedirs(model_dir, exist_ok=True)
    for name, tree in (("actor", actor_reference_tree(algo.actor)), ("Vl", value_reference_tree(algo.Vl)),
                       ("Vh", value_reference_tree(algo.Vh))):
        np.savez(os.path.join(model_dir, f"{name}.npz"), **flatten(tree))

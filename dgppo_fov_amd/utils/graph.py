"""Batched graph container with the reference's field order (dgppo/utils/graph.py:47-189).

The reference's GraphsTuple is a JAX pytree of ONE graph that `jax.vmap` batches.  Here every
field carries explicit leading batch dims (B,) or (B, T) and lives in HBM as a dense padded
tensor; node_type / n_node / n_edge are static per env config and are stride-0 expanded views.
"""
from __future__ import annotations

from typing import Any, NamedTuple, Optional

import torch


class GraphsTuple(NamedTuple):
    n_node: torch.Tensor  # (...,) int32
    n_edge: torch.Tensor  # (...,) int32
    nodes: torch.Tensor  # (..., N, node_dim)
    edges: torch.Tensor  # (..., E, edge_dim)
    states: torch.Tensor  # (..., N, state_dim)
    receivers: torch.Tensor  # (..., E) int32
    senders: torch.Tensor  # (..., E) int32
    node_type: torch.Tensor  # (..., N) int32; 0 agent, 1 goal, 2 obstacle / lidar hit, -1 pad
    env_states: Any
    connectivity: Optional[torch.Tensor] = None

    @property
    def is_single(self) -> bool:
        return self.n_node.dim() == 0

    @property
    def n_graphs(self) -> int:
        return 1 if self.n_node.dim() == 0 else int(self.n_node.numel())

    @property
    def batch_shape(self):
        return tuple(self.n_node.shape)

    def _type_rows(self, type_idx: int, n_type: int) -> torch.Tensor:
        nt = self.node_type
        if nt.dim() > 1:
            nt = nt.reshape(-1, nt.shape[-1])[0]
        ids = torch.nonzero(nt == type_idx).flatten()
        return ids[:n_type]

    def type_nodes(self, type_idx: int, n_type: int) -> torch.Tensor:
        """Rows of one node type (graph.py:115-127): (..., n_type, node_dim)."""
        return self.nodes.index_select(-2, self._type_rows(type_idx, n_type).to(self.nodes.device))

    def type_states(self, type_idx: int, n_type: int) -> torch.Tensor:
        """States of one node type (graph.py:129-141): (..., n_type, state_dim)."""
        return self.states.index_select(-2, self._type_rows(type_idx, n_type).to(self.states.device))

    def without_edge(self) -> "GraphsTuple":
        return self._replace(edges=None)


def tree_map(fn, tree):
    """Map over the tensor leaves of GraphsTuple / NamedTuple env states."""
    if tree is None:
        return None
    if isinstance(tree, torch.Tensor):
        return fn(tree)
    if hasattr(tree, "_map_tensors"):
        return tree._map_tensors(fn)
    if isinstance(tree, tuple) and hasattr(tree, "_fields"):
        return type(tree)(*[tree_map(fn, x) for x in tree])
    if isinstance(tree, (list, tuple)):
        return type(tree)(tree_map(fn, x) for x in tree)
    if isinstance(tree, dict):
        return {k: tree_map(fn, v) for k, v in tree.items()}
    return tree


def tree_index(tree, idx):
    return tree_map(lambda x: x[idx], tree)

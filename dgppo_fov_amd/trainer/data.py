"""Rollout container (dgppo/trainer/data.py:8-32) with leading (B, T) dims.

`graph` and `next_graph` are two views of ONE (B, T+1, ...) buffer (graph = [:, :T], next_graph =
[:, 1:]); the reference stores both, doubling the rollout's HBM footprint."""
from typing import NamedTuple, Optional

import torch

from ..utils.graph import GraphsTuple


class Rollout(NamedTuple):
    graph: GraphsTuple
    actions: torch.Tensor  # (B, T, n, 2)
    rnn_states: Optional[torch.Tensor]  # (B, T, rnn_layers, n, carries, 64) actor carries
    rewards: torch.Tensor  # (B, T)
    costs: torch.Tensor  # (B, T, n, n_cost)
    dones: torch.Tensor  # (B, T) bool
    log_pis: Optional[torch.Tensor]  # (B, T, n)
    next_graph: GraphsTuple

    @property
    def length(self) -> int:
        return self.rewards.shape[0]

    @property
    def time_horizon(self) -> int:
        return self.rewards.shape[1]

    @property
    def num_agents(self) -> int:
        return self.costs.shape[2]

    @property
    def n_data(self) -> int:
        return self.length * self.time_horizon

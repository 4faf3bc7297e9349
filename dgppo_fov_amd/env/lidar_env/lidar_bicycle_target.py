"""LidarBicycleTarget (dgppo/env/lidar_env/lidar_bicycle_target.py:23-123): kinematic bicycle
agents, state [x, y, cos th, sin th, v], edge features [x, y, v cos th, v sin th]."""
import math

import torch

from ... import _lib
from .lidar_target import LidarTarget


class LidarBicycleTarget(LidarTarget):
    ENGINE = _lib.DGPPO_ENGINE_BICYCLE
    PARAMS = dict(LidarTarget.PARAMS)

    @property
    def state_dim(self) -> int:
        return 5  # x, y, cos(theta), sin(theta), v

    @property
    def node_dim(self) -> int:
        return 8

    def state_lim(self, state=None):
        a = self.area_size
        return torch.tensor([0.0, 0.0, -1.0, -1.0, -0.5]), torch.tensor([a, a, 1.0, 1.0, 0.5])

    def _obs_theta_range(self):
        return -math.pi, math.pi  # lidar_bicycle_target.py:76

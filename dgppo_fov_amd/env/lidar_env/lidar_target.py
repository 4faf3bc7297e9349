"""LidarTarget (dgppo/env/lidar_env/lidar_target.py): agent i is wired to and rewarded by goal i
(DGPPO_GOAL_TARGET)."""
from ... import _lib
from .base import LidarEnv


class LidarTarget(LidarEnv):
    GOAL_MODE = _lib.DGPPO_GOAL_TARGET
    PARAMS = dict(LidarEnv.PARAMS)

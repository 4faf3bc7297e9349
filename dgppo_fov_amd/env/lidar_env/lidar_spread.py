"""LidarSpread (dgppo/env/lidar_env/lidar_spread.py): each goal rewards its nearest agent; every
agent is wired to every goal (DGPPO_GOAL_SPREAD)."""
from ... import _lib
from .base import LidarEnv


class LidarSpread(LidarEnv):
    GOAL_MODE = _lib.DGPPO_GOAL_SPREAD
    PARAMS = dict(LidarEnv.PARAMS)

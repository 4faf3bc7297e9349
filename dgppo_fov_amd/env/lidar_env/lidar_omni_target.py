"""LidarOmniTarget (dgppo/env/lidar_env/lidar_omni_target.py): omni-wheel (mecanum) agents that
must keep agent i+1 inside agent i's field of view.

State [x, y, cos th, sin th, vx, vy, omega] (7), action [ax, ay, alpha] (3, alpha limited to
+-1000), node features state + 3 indicators (10), edge features 10: [s_i - s_j (7) | critical
edge i -> i+1 | ||p_j^i|| | i_x_j] with p_j^i = R_i^T (p_j - p_i) the receiver-frame offset.
Five costs: agent collision, obstacle collision, and on the chain i -> i+1 the FoV angle,
maximum range and minimum distance (lidar_omni_target.py:517-649).  Reset places agents with
min distance max(2.2 r, D) and points agent i at agent i+1.  Step / reset run in
libdgppo_hip.so (omni_step_kernel / env_reset_kernel)."""
from typing import Tuple

import torch

from ... import _lib
from .lidar_target import LidarTarget


class LidarOmniTarget(LidarTarget):
    ENGINE = _lib.DGPPO_ENGINE_OMNI
    PARAMS = {
        "car_radius": 0.05,
        "comm_radius": 0.5,
        "n_rays": 32,
        "obs_len_range": [0.1, 0.3],
        "n_obs": 3,
        "default_area_size": 1.5,
        "dist2goal": 0.01,
        "top_k_rays": 8,
        "max_angular_vel": 100.0,
        "rotation_penalty": 0.001,
        "fov_angle_deg": 60.0,
        "max_sensor_range": 0.5,
        "min_safe_distance": 0.2,
    }

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        p = self.params
        # lidar_omni_target.py:97-100
        assert p["min_safe_distance"] > 2 * p["car_radius"], "min_safe_distance must exceed 2 * car_radius"
        assert p["min_safe_distance"] < p["max_sensor_range"], "min_safe_distance must be below max_sensor_range"

    # Node columns a goal / lidar-hit node can have nonzero: position (0, 1) and its type one-hot (7, 8);
    # goals are [pos, 0 x 5] (lidar_omni_target.py:281-284), hits [pos, 0 x 5] (lidar_env/base.py get_graph).
    nonagent_feature_cols = (0, 1, 7, 8)

    @property
    def n_cost(self) -> int:
        return 5

    @property
    def cost_components(self) -> Tuple[str, ...]:
        return "agent collisions", "obs collisions", "fov angle", "fov max range", "fov min distance"

    @property
    def state_dim(self) -> int:
        return 7

    @property
    def node_dim(self) -> int:
        return 10

    @property
    def edge_dim(self) -> int:
        return 10

    @property
    def action_dim(self) -> int:
        return 3

    def state_lim(self, state=None):
        a, w = self.area_size, float(self.params["max_angular_vel"])
        return (torch.tensor([0.0, 0.0, -1.0, -1.0, -2.0, -2.0, -w]),
                torch.tensor([a, a, 1.0, 1.0, 2.0, 2.0, w]))

    def action_lim(self):
        return torch.tensor([-1.0, -1.0, -1000.0]), torch.tensor([1.0, 1.0, 1000.0])

    def _engine_cfg(self, c: _lib.EnvCfg) -> None:
        import numpy as np

        p = self.params
        c.omni_max_w = p["max_angular_vel"]
        c.fov_angle_deg = p["fov_angle_deg"]
        c.fov_rmax = p["max_sensor_range"]
        c.fov_dmin = p["min_safe_distance"]
        c.rot_pen = p["rotation_penalty"]
        # reset spacing: jnp.maximum(2.2 r, D) in float32, inside-obstacle radius min_dist / 2
        md = float(max(np.float32(2.2 * p["car_radius"]), np.float32(p["min_safe_distance"])))
        c.c_min_dist = md
        c.c_inside_r = float(np.float32(np.float32(md) / np.float32(2)))

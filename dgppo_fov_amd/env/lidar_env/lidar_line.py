"""LidarLine (dgppo/env/lidar_env/lidar_line.py): LidarSpread with TWO landmark goal nodes; the n reward
goals are the evenly spaced points of the segment between them (landmark2goal, :137-142), and the reset
places the landmarks and the rectangle obstacles by rejection (:38-126).  Step/reset: the variant kernels
of libdgppo_hip.so (DGPPO_VARIANT_LINE)."""
from ... import _lib
from .lidar_spread import LidarSpread


class LidarLine(LidarSpread):
    PARAMS = dict(LidarSpread.PARAMS)

    def __init__(self, num_agents, area_size=None, max_step=128, dt=0.03, params=None, device=None):
        area = type(self).PARAMS["default_area_size"] if area_size is None else area_size
        p = type(self).PARAMS if params is None else params
        if area - (num_agents - 2) * 6 * p["car_radius"] < 0:  # lidar_line.py:56-58
            raise ValueError("The area size is too small to place the landmarks.")
        super().__init__(num_agents, area_size, max_step, dt, params, device)

    def _n_goals(self) -> int:
        return 2

    def _engine_cfg(self, c) -> None:
        r, area = self._params["car_radius"], self._area_size
        md = (self._num_agents - 2) * 6 * r
        side = area - md
        c.variant = _lib.DGPPO_VARIANT_LINE
        c.line_min_dist = md
        c.line_box_x, c.line_box_y, c.line_off_y = area - side, side, area / 2 - side
        c.c_obs_inflate = r * 1.1

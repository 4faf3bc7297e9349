"""MPETarget (dgppo/env/mpe/mpe_target.py).  With obs=0 the reference crashes in edge_blocks
(`None[:, :2]`, mpe_target.py:72 via mpe/base.py:143); here an empty obstacle block is used, so
the obstacle cost is 0 - 0.5 = -0.5 (the natural semantics)."""
from ... import _lib
from .base import MPE


class MPETarget(MPE):
    GOAL_MODE = _lib.DGPPO_GOAL_TARGET
    PARAMS = dict(MPE.PARAMS)

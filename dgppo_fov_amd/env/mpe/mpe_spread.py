"""MPESpread (dgppo/env/mpe/mpe_spread.py)."""
from ... import _lib
from .base import MPE


class MPESpread(MPE):
    GOAL_MODE = _lib.DGPPO_GOAL_SPREAD
    PARAMS = dict(MPE.PARAMS)

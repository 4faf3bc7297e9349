from .base import MPE, MPEEnvState
from .mpe_spread import MPESpread
from .mpe_target import MPETarget
from .mpe_variants import MPEConnectSpread, MPECorridor, MPEFormation, MPELine

"""Env registry + make_env (dgppo/env/__init__.py:10-55).

Every env of the reference is built: Lidar and MPE (the variants LidarLine, MPELine, MPEFormation,
MPECorridor and MPEConnectSpread on the variant kernels) and the two VMAS contact-physics envs
(csrc/vmas.hip), SURVEY.md §8f rank 4."""
from typing import Optional

from .base import MultiAgentEnv, StepResult, RolloutResult
from .lidar_env import (LidarSpread, LidarTarget, LidarBicycleTarget, LidarOmniTarget, LidarLine, LidarEnv,
                        LidarEnvState)
from .mpe import (MPESpread, MPETarget, MPELine, MPEFormation, MPECorridor, MPEConnectSpread, MPE,
                  MPEEnvState)
from .vmas import VMASWheel, VMASReverseTransport, VMASEnv

ENV = {
    "MPETarget": MPETarget,
    "MPESpread": MPESpread,
    "MPELine": MPELine,
    "MPEFormation": MPEFormation,
    "MPECorridor": MPECorridor,
    "MPEConnectSpread": MPEConnectSpread,
    "LidarSpread": LidarSpread,
    "LidarTarget": LidarTarget,
    "LidarLine": LidarLine,
    "LidarBicycleTarget": LidarBicycleTarget,
    "LidarOmniTarget": LidarOmniTarget,
    "VMASReverseTransport": VMASReverseTransport,
    "VMASWheel": VMASWheel,
}

DEFAULT_MAX_STEP = 128


def make_env(env_id: str, num_agents: int, max_step: int = None, full_observation: bool = False,
             num_obs: Optional[int] = None, n_rays: Optional[int] = None, device=None) -> MultiAgentEnv:
    assert env_id in ENV, f"Environment {env_id} not implemented."
    params = dict(ENV[env_id].PARAMS)  # copied: the reference mutates the class dict (env/__init__.py:40-46)
    max_step = DEFAULT_MAX_STEP if max_step is None else max_step
    if num_obs is not None:
        params["n_obs"] = num_obs
    if n_rays is not None:
        params["n_rays"] = n_rays
    if full_observation:
        area_size = params["default_area_size"]
        params["comm_radius"] = area_size * 10
    return ENV[env_id](num_agents=num_agents, area_size=None, max_step=max_step, dt=0.03, params=params,
                       device=device)

"""Env registry + make_env (dgppo/env/__init__.py:10-55).

Only the engines BASELINE.json's configs use are built; the other reference
variants (MPEFormation/Line/Corridor/ConnectSpread, LidarLine, LidarOmniTarget, VMAS) are listed
in DESIGN.md as next rows and raise here."""
from typing import Optional

from .base import MultiAgentEnv, StepResult, RolloutResult
from .lidar_env import LidarSpread, LidarTarget, LidarBicycleTarget, LidarEnv, LidarEnvState
from .mpe import MPESpread, MPETarget, MPE, MPEEnvState

ENV = {
    "MPETarget": MPETarget,
    "MPESpread": MPESpread,
    "LidarSpread": LidarSpread,
    "LidarTarget": LidarTarget,
    "LidarBicycleTarget": LidarBicycleTarget,
}

NOT_YET_BUILT = ("MPELine", "MPEFormation", "MPECorridor", "MPEConnectSpread", "LidarLine",
                 "LidarOmniTarget", "VMASReverseTransport", "VMASWheel")

DEFAULT_MAX_STEP = 128


def make_env(env_id: str, num_agents: int, max_step: int = None, full_observation: bool = False,
             num_obs: Optional[int] = None, n_rays: Optional[int] = None, device=None) -> MultiAgentEnv:
    if env_id in NOT_YET_BUILT:
        raise NotImplementedError(f"Environment {env_id} is not built yet (see DESIGN.md, next rows)")
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

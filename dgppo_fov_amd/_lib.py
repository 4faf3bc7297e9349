"""ctypes binding of libdgppo_hip.so (include/dgppo_hip.h).

The product path has exactly one implementation — the HIP kernels in this library.  If the
library is missing or cannot be loaded, every op raises `NativeLibraryError`; there is no CPU or
PyTorch fallback.
"""
from __future__ import annotations

import ctypes
import os
import pathlib

PKG_DIR = pathlib.Path(__file__).resolve().parent
LIB_PATH = pathlib.Path(os.environ.get("DGPPO_HIP_LIB", PKG_DIR / "lib" / "libdgppo_hip.so"))

DGPPO_EINVAL = -22
DGPPO_ENGINE_LIDAR, DGPPO_ENGINE_BICYCLE, DGPPO_ENGINE_MPE = 0, 1, 2
DGPPO_GOAL_SPREAD, DGPPO_GOAL_TARGET = 0, 1
DGPPO_OBST_FIELDS = 16

c_f32p = ctypes.c_void_p  # device pointers travel as raw addresses


class NativeLibraryError(RuntimeError):
    pass


class EnvCfg(ctypes.Structure):
    _fields_ = [
        ("engine", ctypes.c_int32),
        ("goal_mode", ctypes.c_int32),
        ("n_agents", ctypes.c_int32),
        ("n_obs", ctypes.c_int32),
        ("n_rays", ctypes.c_int32),
        ("top_k", ctypes.c_int32),
        ("state_dim", ctypes.c_int32),
        ("node_dim", ctypes.c_int32),
        ("n_nodes", ctypes.c_int32),
        ("n_edges", ctypes.c_int32),
        ("dt", ctypes.c_float),
        ("comm_radius", ctypes.c_float),
        ("car_radius", ctypes.c_float),
        ("obs_radius", ctypes.c_float),
        ("area_size", ctypes.c_float),
        ("dist2goal", ctypes.c_float),
        ("obs_len_lo", ctypes.c_float),
        ("obs_len_hi", ctypes.c_float),
        ("obs_theta_lo", ctypes.c_float),
        ("obs_theta_hi", ctypes.c_float),
        ("state_lo", ctypes.c_float * 5),
        ("state_hi", ctypes.c_float * 5),
        ("c_agent_cost", ctypes.c_float),
        ("c_obs_cost", ctypes.c_float),
        ("c_self_dist", ctypes.c_float),
        ("c_lidar_active", ctypes.c_float),
        ("c_min_dist", ctypes.c_float),
        ("c_inside_r", ctypes.c_float),
        ("c_mpe_obs_agent", ctypes.c_float),
        ("c_mpe_obs_goal", ctypes.c_float),
        ("c_mpe_obs_lo", ctypes.c_float),
        ("c_mpe_obs_hi", ctypes.c_float),
    ]


class EnvStepIO(ctypes.Structure):
    _fields_ = [
        ("states", c_f32p), ("states_stride", ctypes.c_int64),
        ("obstacles", c_f32p), ("obstacles_stride", ctypes.c_int64),
        ("action", c_f32p), ("action_stride", ctypes.c_int64),
        ("ray_dirs", c_f32p),
        ("nodes", c_f32p), ("nodes_stride", ctypes.c_int64),
        ("edges", c_f32p), ("edges_stride", ctypes.c_int64),
        ("out_states", c_f32p), ("out_states_stride", ctypes.c_int64),
        ("receivers", c_f32p), ("senders", c_f32p), ("edge_index_stride", ctypes.c_int64),
        ("reward", c_f32p), ("reward_stride", ctypes.c_int64),
        ("cost", c_f32p), ("cost_stride", ctypes.c_int64),
        ("n_env", ctypes.c_int32),
    ]


class EnvResetIO(ctypes.Structure):
    _fields_ = [
        ("seed", ctypes.c_uint64),
        ("seed_ptr", c_f32p),
        ("env_offset", ctypes.c_int32),
        ("obstacles", c_f32p), ("obstacles_stride", ctypes.c_int64),
        ("ray_dirs", c_f32p),
        ("nodes", c_f32p), ("nodes_stride", ctypes.c_int64),
        ("edges", c_f32p), ("edges_stride", ctypes.c_int64),
        ("out_states", c_f32p), ("out_states_stride", ctypes.c_int64),
        ("receivers", c_f32p), ("senders", c_f32p), ("edge_index_stride", ctypes.c_int64),
        ("n_env", ctypes.c_int32),
    ]


# symbol -> (restype, argtypes); must match include/dgppo_hip.h (checked by tests/test_capi.py)
SIGNATURES = {
    "dgppo_abi_version": (ctypes.c_int, []),
    "dgppo_build_info": (ctypes.c_char_p, []),
    "dgppo_env_cfg_finalize": (ctypes.c_int, [ctypes.POINTER(EnvCfg)]),
    "dgppo_ray_table": (ctypes.c_int, [ctypes.c_int32, ctypes.c_float, ctypes.c_void_p]),
    "dgppo_env_step": (ctypes.c_int, [ctypes.POINTER(EnvCfg), ctypes.POINTER(EnvStepIO), ctypes.c_void_p]),
    "dgppo_env_reset": (ctypes.c_int, [ctypes.POINTER(EnvCfg), ctypes.POINTER(EnvResetIO), ctypes.c_void_p]),
}

_LIB = None


def load() -> ctypes.CDLL:
    """Load the HIP library once (torch must be imported first so one HIP runtime is shared)."""
    global _LIB
    if _LIB is not None:
        return _LIB
    import torch  # noqa: F401  (loads torch's libamdhip64.so.7 first; ours binds to the same soname)

    if not LIB_PATH.exists():
        raise NativeLibraryError(
            f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` or `make`"
        )
    try:
        lib = ctypes.CDLL(str(LIB_PATH), mode=ctypes.RTLD_GLOBAL)
    except OSError as e:  # pragma: no cover
        raise NativeLibraryError(f"cannot load {LIB_PATH}: {e}") from e
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _LIB = lib
    return lib


def check(rc: int, what: str):
    if rc == DGPPO_EINVAL:
        raise ValueError(f"{what}: invalid arguments (DGPPO_EINVAL)")
    if rc != 0:
        raise RuntimeError(f"{what}: HIP error {rc}")


def ptr(t) -> int:
    return 0 if t is None else int(t.data_ptr())


def stream_handle(device=None) -> int:
    import torch

    return int(torch.cuda.current_stream(device).cuda_stream)


def require_gpu(device, what: str):
    """The kernels only run on the GPU; there is deliberately no CPU path."""
    import torch

    if torch.device(device).type != "cuda":
        raise NativeLibraryError(f"{what}: libdgppo_hip kernels need GPU tensors (got device {device})")

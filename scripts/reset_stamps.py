"""Phase timers of the env reset kernel (diagnostic library: a copy of csrc/env_step.hip with s_memtime stamps in
env_reset_kernel, compiled with -DDGPPO_ENV_STAMPS into dgppo_fov_amd/lib/libdgppo_hip_rdiag.so; the shipped sources
carry no stamps).  Prints thread 0's ticks per env and phase, averaged over the resets.
Usage: DGPPO_HIP_LIB=dgppo_fov_amd/lib/libdgppo_hip_rdiag.so python scripts/reset_stamps.py ENV n obs B [states]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from dgppo_fov_amd import _lib  # noqa: E402
from dgppo_fov_amd.env import make_env  # noqa: E402

PHASES = ["obstacles", "candidate table", "rejection sampler", "rows", "MPE obstacles / omni headings",
          "bicycle headings", "-", "graph write"]


def main():
    eid, n, obs, B = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    states = len(sys.argv) > 5 and sys.argv[5] == "states"
    dev = torch.device("cuda:0")
    env = make_env(eid, n, num_obs=obs, device=dev)
    fn = _lib.load().dgppo_env_diag_stamps
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
    buf = (ctypes.c_ulonglong * 16)()
    g = env.reset_states(1, n_env=B) if states else env.reset(1, n_env=B)
    torch.cuda.synchronize()
    fn(buf)
    reps = 10
    for i in range(reps):
        if states:
            env.reset_states(100 + i, n_env=B, out=g)
        else:
            env.reset(100 + i, n_env=B)
    torch.cuda.synchronize()
    fn(buf)
    per = {PHASES[k]: round(buf[k] / (reps * B), 1) for k in range(8) if buf[k]}
    print(json.dumps({"env": eid, "n": n, "obs": obs, "envs": B, "states_only": states,
                      "ticks_per_env": per, "total": round(sum(buf[k] for k in range(8)) / (reps * B), 1)}))


if __name__ == "__main__":
    main()

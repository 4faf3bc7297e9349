"""Phase timers of the persistent env rollout (diagnostic library, `make stamps`): per wave and step, the
s_memtime ticks spent in each phase of wv::wave_body, averaged over the timed launches.
Run with DGPPO_HIP_LIB=dgppo_fov_amd/lib/libdgppo_hip_stamps.so (set below when unset)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("DGPPO_HIP_LIB", os.path.join(ROOT, "dgppo_fov_amd", "lib", "libdgppo_hip_stamps.so"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from dgppo_fov_amd import _lib  # noqa: E402
from dgppo_fov_amd.env import make_env  # noqa: E402
from dgppo_fov_amd.trainer.rollout import RolloutEngine  # noqa: E402

PHASES = ["A: action, LDS staging", "B: dynamics, distances", "C: cost, reward", "F1 packet 1 (agent-agent edges)",
          "D: is-inside, culling masks", "packet 2 (agent-goal edges)", "capsule tests, item list",
          "packet 3 (agent/goal node+state rows)", "barrier 1 wait", "pooled ray cast", "packet 4 (hit-row constants)",
          "barrier 2 wait", "E: sort keys, miss ranks", "E: ranks of the hits", "F2: lidar columns"]


def main():
    eid = sys.argv[1] if len(sys.argv) > 1 else "LidarSpread"
    B, T, reps = 4096, 128, 5
    dev = torch.device("cuda:0")
    env = make_env(eid, 8, num_obs=3, device=dev)
    eng = RolloutEngine(env, B, T, dev, lanes=1)
    eng.actions.uniform_(-1.0, 1.0)
    lib = _lib.load()
    fn = lib.dgppo_env_diag_stamps
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
    buf = (ctypes.c_ulonglong * 16)()
    eng.run(key=0)
    torch.cuda.synchronize()
    fn(buf)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for k in range(reps):
        eng.run(key=1 + k)
    e1.record()
    torch.cuda.synchronize()
    fn(buf)
    per = [buf[k] / (reps * B * T) for k in range(len(PHASES))]  # ticks per wave and step
    tot = sum(per)
    ep = e0.elapsed_time(e1) / reps
    out = {"env": eid, "episode_ms": ep, "ticks_per_wave_step": round(tot, 2),
           "us_per_step": round(ep * 1e3 / T, 3), "ticks_per_us": round(tot / (ep * 1e3 / T), 1),
           "phases": {p: {"ticks": round(v, 2), "frac": round(v / tot, 3)} for p, v in zip(PHASES, per)}}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

"""Phase timers of the workgroup-per-env step kernel (diagnostic library, `make stamps`): wave 0's
barrier-to-barrier s_memtime ticks per env step, for one config (default LidarSpread n=32 o=8, 1024 envs).
Usage: DGPPO_HIP_LIB=dgppo_fov_amd/lib/libdgppo_hip_stamps.so python scripts/block_stamps.py [env n obs B]"""
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

PHASES = ["A: stage rows", "B: dynamics + distance tasks", "C: row minima, cost/reward terms, is-inside",
          "D: reward/cost stores + ray scan + top-k", "E: write the graph"]


def main():
    a = sys.argv[1:]
    eid, n, obs, B = (a[0], int(a[1]), int(a[2]), int(a[3])) if len(a) == 4 else ("LidarSpread", 32, 8, 1024)
    dev = torch.device("cuda:0")
    env = make_env(eid, n, num_obs=obs, device=dev)
    g = env.reset(key=1, n_env=B)
    act = torch.rand(B, n, env.action_dim, device=dev) * 2 - 1
    outs = [env.empty_graph((B,), dev) for _ in range(2)]
    ob = g.env_states.obstacle.packed if hasattr(g.env_states, "obstacle") and g.env_states.obstacle is not None else None
    outs = [env._assemble(o.nodes, o.edges, o.states, o.receivers, o.senders, ob) for o in outs]
    rew = torch.empty(B, device=dev)
    cost = torch.empty(B, n, env.n_cost, device=dev)
    fn = _lib.load().dgppo_env_diag_block_stamps
    fn.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
    buf = (ctypes.c_ulonglong * 8)()
    steps = 32
    cur = env.step_into(g, act, outs[0], rew, cost)
    torch.cuda.synchronize()
    fn(buf)
    for i in range(steps):
        cur = env.step_into(cur, act, outs[(i + 1) & 1], rew, cost)
    torch.cuda.synchronize()
    fn(buf)
    per = [buf[k] / (steps * B) for k in range(len(PHASES))]
    tot = sum(per)
    print(json.dumps({"env": eid, "n": n, "obs": obs, "B": B, "ticks_per_env_step": round(tot, 1),
                      "phases": {p: {"ticks": round(v, 1), "frac": round(v / tot, 3)} for p, v in zip(PHASES, per)}},
                     indent=1))


if __name__ == "__main__":
    main()

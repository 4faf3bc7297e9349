"""Per-kernel cost of each network pass on one DGPPO minibatch (LidarSpread n8, 16384 graphs =
1024 sequences x 16 steps).  Phases are separated by idle gaps so a kernel trace can be split:
run under `rocprofv3 --kernel-trace --output-format csv` and post-process with --split <trace.csv>."""
import csv
import os
import sys
import time
from collections import defaultdict

PH = ["Vl_fwd", "Vl_bwd", "Vh_fwd", "Vh_bwd", "pi_fwd", "pi_bwd"]

if len(sys.argv) > 2 and sys.argv[1] == "--split":
    rows = sorted(csv.DictReader(open(sys.argv[2])), key=lambda r: int(r["Start_Timestamp"]))
    groups, cur, last = [], [], None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if last is not None and s - last > 20_000_000:  # 20 ms gap
            groups.append(cur)
            cur = []
        cur.append(r)
        last = e
    groups.append(cur)
    groups = groups[-len(PH):]
    for name, g in zip(PH, groups):
        agg = defaultdict(lambda: [0, 0.0])
        for r in g:
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-50:]
            agg[k][0] += 1
            agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot = sum(v[1] for v in agg.values()) / REPS if (REPS := 5) else 0
        print(f"== {name}: {tot:.1f} us per pass ({len(g) // REPS} kernels)")
        for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:12]:
            print(f"   {v[1] / REPS:9.1f} us  x{v[0] // REPS:3d}  {k}")
    sys.exit(0)

import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgppo_fov_amd.algo import make_algo  # noqa: E402
from dgppo_fov_amd.env import make_env  # noqa: E402
from dgppo_fov_amd.nn import kernels as K  # noqa: E402

dev = torch.device("cuda:0")
# MB_ENV / MB_N / MB_OBS pick another config (e.g. the dense LidarSpread n=32, 8 obstacles)
EID, n, OBS = os.environ.get("MB_ENV", "LidarSpread"), int(os.environ.get("MB_N", 8)), int(os.environ.get("MB_OBS", 3))
T, B = 128, 1024
env = make_env(EID, n, num_obs=OBS, max_step=T, device=dev)
algo = make_algo("dgppo", env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                 action_dim=env.action_dim, n_agents=n, batch_size=16384, device=dev, train_steps=100)
r = algo.collect(algo.params, 0, n_env=B)
envs = torch.arange(128, device=dev)
g = algo._graphs(r.graph, envs)
S, L = 128 * T // 16, 16
acts = r.actions.index_select(0, envs).reshape(-1, env.action_dim).contiguous()
hd = r.rnn_states.index_select(0, envs).reshape(-1, 64).contiguous()
REPS = 5


def phase(fn):
    torch.cuda.synchronize()
    time.sleep(0.05)
    for _ in range(REPS):
        fn()
    torch.cuda.synchronize()


state = {}


def vl_f():
    v, _, c = algo.Vl.seq_fwd(g, S, L)
    state["vl"] = (v, c)


def vl_b():
    v, c = state["vl"]
    algo.Vl.seq_bwd(c, torch.ones_like(v) * 1e-4)


def vh_f():
    state["vh"] = algo.Vh.fwd(g, hd)


def vh_b():
    o, c = state["vh"]
    algo.Vh.bwd(c, torch.ones_like(o) * 1e-4)


def pi_f():
    state["pi"] = algo.actor.eval_seq_fwd(g, S, L, acts, algo.entropy_eps)


def pi_b():
    lp, ent, c = state["pi"]
    algo.actor.eval_seq_bwd(c, torch.ones_like(lp) * 1e-4, torch.ones_like(ent) * 1e-4)


vl_f(), vl_b(), vh_f(), vh_b(), pi_f(), pi_b()  # warm
for fn in (vl_f, vl_b, vh_f, vh_b, pi_f, pi_b):
    t0 = time.perf_counter()
    phase(fn)
    print(f"{fn.__name__}: {(time.perf_counter() - t0 - 0.05) / REPS * 1e3:.2f} ms/pass (host incl.)", flush=True)

"""Per-shape GEMM time of one DGPPO update at the bench config: run under
`rocprofv3 --kernel-trace --output-format csv -d DIR -o upd`, then
`python scripts/gemm_time_by_shape.py --analyze DIR/upd_kernel_trace.csv gemm_log.json`.
The n-th dgppo_gemm call's kernels (main + optional reduce) are matched to the n-th GEMM_LOG entry."""
import collections
import csv
import json
import os
import sys

if len(sys.argv) > 1 and sys.argv[1] == "--analyze":
    rows = sorted(csv.DictReader(open(sys.argv[2])), key=lambda r: int(r["Start_Timestamp"]))
    log = json.load(open(sys.argv[3]))
    ks = [r for r in rows if "gemm" in r["Kernel_Name"]]
    # keep only the logged update: the last len(log) main launches
    mains = [r for r in ks if "reduce" not in r["Kernel_Name"]]
    mains = mains[-len(log):]
    agg = collections.defaultdict(lambda: [0, 0.0, ""])
    for r, e in zip(mains, log):
        key = tuple(e)
        a = agg[key]
        a[0] += 1
        a[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        a[2] = r["Kernel_Name"].split("(")[0].replace("void dgppo::", "")
    tot = sum(v[1] for v in agg.values())
    print(f"{len(log)} GEMM calls, {tot / 1e3:.1f} ms")
    for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:30]:
        M, N, Kd, b, ta, tb, sk, bias = k
        byt = 4 * (M * Kd + Kd * N + M * N) * b
        print(f"{v[1] / 1e3:7.2f} ms n={v[0]:4d} avg {v[1] / v[0]:7.1f} us  M={M} N={N} K={Kd} b={b} ta={ta} tb={tb} "
              f"{v[2]:28s} {byt / (v[1] / v[0]) / 1e3:6.0f} GB/s")
    sys.exit(0)

import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dgppo_fov_amd.algo import make_algo  # noqa: E402
from dgppo_fov_amd.env import make_env  # noqa: E402
from dgppo_fov_amd.nn import kernels as K  # noqa: E402

dev = torch.device("cuda:0")
env = make_env("LidarSpread", 8, num_obs=3, device=dev)
algo = make_algo("dgppo", env=env, node_dim=env.node_dim, edge_dim=env.edge_dim, state_dim=env.state_dim,
                 action_dim=env.action_dim, n_agents=8, batch_size=16384, device=dev, train_steps=100)
r = algo.collect(algo.params, 0, n_env=4096)
algo.update(r, 0)
torch.cuda.synchronize()
K.GEMM_LOG = []
algo.update(r, 1)
torch.cuda.synchronize()
json.dump(K.GEMM_LOG, open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/gemm_log.json", "w"))
print("logged", len(K.GEMM_LOG))

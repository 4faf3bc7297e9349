"""Kernels of the last update in a rocprofv3 --kernel-trace CSV (scripts/update_time.py --reps 1 under tracing):
count, total and mean duration per kernel name, per minibatch (argv[2] = minibatches per update), largest first."""
import csv
import glob
import sys
from collections import defaultdict

fn = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
nmb = int(sys.argv[2]) if len(sys.argv) > 2 else 32
rs = sorted(csv.DictReader(open(fn)), key=lambda r: int(r["Start_Timestamp"]))
w = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].replace("(anonymous namespace)::", "")
      .split("(")[0][-60:]) for r in rs]
last_pol = max(i for i, x in enumerate(w) if "policy_step" in x[2] or "rollout" in x[2])
w = w[last_pol + 1:]
agg = defaultdict(lambda: [0, 0])
for s, e, k in w:
    agg[k][0] += 1
    agg[k][1] += e - s
tot = sum(v[1] for v in agg.values())
print(f"{len(w)} kernels, {tot / 1e6:.2f} ms summed; per minibatch ({nmb}): {len(w) / nmb:.1f} kernels")
for k, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:40]:
    print(f"{t / 1e3:9.1f} us {100 * t / tot:5.1f}%  n={n:5d} ({n / nmb:5.1f}/mb)  mean {t / n / 1e3:7.2f} us  {k}")

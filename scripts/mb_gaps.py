"""Idle time of the GPU inside the last update of a rocprofv3 kernel trace (scripts/update_time.py --reps 1 under
--kernel-trace): union of kernel intervals vs the update window, and the largest idle gaps by kernel transition."""
import csv
import glob
import sys
from collections import Counter

fn = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rs = sorted(csv.DictReader(open(fn)), key=lambda r: int(r["Start_Timestamp"]))
w = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"],
      r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-42:]) for r in rs]
# the last update: from the last gather_env_steps after the last policy_step (collect) to the end
last_pol = max(i for i, x in enumerate(w) if "policy_step" in x[3] or "lidar_step" in x[3] or "rollout" in x[3])
w = w[last_pol + 1:]
t0, t1 = w[0][0], max(x[1] for x in w)
busy, cs, ce, last, lastk, gaps = 0, None, None, None, None, Counter()
cnt = Counter()
for s, e, q, k in w:
    if ce is None or s > ce:
        if ce is not None:
            busy += ce - cs
            gaps[(lastk, k)] += s - ce
            cnt[(lastk, k)] += 1
        cs, ce = s, e
    else:
        ce = max(ce, e)
    if last is None or e >= last:
        last, lastk = e, k
busy += ce - cs
print(f"window {(t1 - t0) / 1e6:.2f} ms  busy {busy / 1e6:.2f} ms  idle {(t1 - t0 - busy) / 1e6:.2f} ms  kernels {len(w)} "
      f"queues {sorted(Counter(x[2] for x in w).items())}")
for key, v in gaps.most_common(10):
    print(f"  {v / 1e3:8.1f} us n={cnt[key]:3d}  {key[0]} -> {key[1]}")

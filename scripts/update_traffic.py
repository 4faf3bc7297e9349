"""Join scripts/update_traffic_pmc.sh's passes: per kernel family, HBM bytes of ONE DGPPO update (the dispatches
after the last `spin_kernel` marker of update_smoke.py) as 2 x FETCH_SIZE + WRITE_SIZE (gfx950 correction for
16-byte streaming reads; other access widths are uncalibrated, so narrow gathers may be under-counted), the
family's kernel time in the un-instrumented trace's update window and the implied GB/s."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def family(name):
    n = name.replace("(anonymous namespace)::", "")
    m = re.search(r"(gemm_rows\w*?_kernel|gemm_wgrad_reduce|gemm_wgrad_kernel|gemm_kernel|attn_\w+?_kernel|"
                  r"gru_seq_\w+?_kernel|policy_step_kernel|lidar_\w+?_kernel|layernorm64_\w+?_kernel|gae_kernel|"
                  r"adam_kernel|colsum_\w+?_kernel|relu_bwd_kernel|gather_env_steps_kernel|sender_table_kernel|"
                  r"elementwise_kernel|FillFunctor|\w+_kernel)", n)
    return m.group(1) if m else "other"

root = sys.argv[1]


def rows(sub, name):
    return list(csv.DictReader(open(glob.glob(os.path.join(root, sub, "**", name), recursive=True)[0])))


def after_mark(rs, key):
    marks = [int(r[key]) for r in rs if "spin_kernel" in r["Kernel_Name"]]
    return [r for r in rs if int(r[key]) > max(marks)]


out = {"window": "one DGPPO update after the second collect (update_smoke.py, LidarSpread n8 o3, 4096 envs, "
                 "batch 16384: prepass + 32 minibatches)", "families": {}}
by = defaultdict(lambda: defaultdict(float))
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    pr = after_mark(rows(c, "*counter_collection.csv"), "Dispatch_Id")
    for r in pr:
        if r["Counter_Name"] == c:
            by[family(r["Kernel_Name"])][c] += float(r["Counter_Value"]) * 1024.0  # counters report KB
tr = rows("trace", "*kernel_trace.csv")
marks = [int(r["End_Timestamp"]) for r in tr if "spin_kernel" in r["Kernel_Name"]]
upd = [r for r in tr if int(r["Start_Timestamp"]) >= max(marks)]
dur = defaultdict(float)
for r in upd:
    dur[family(r["Kernel_Name"])] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
span = (max(int(r["End_Timestamp"]) for r in upd) - min(int(r["Start_Timestamp"]) for r in upd)) * 1e-9
tot = 0.0
for fam in sorted(set(by) | set(dur), key=lambda f: -(2 * by[f]["FETCH_SIZE"] + by[f]["WRITE_SIZE"])):
    b = 2 * by[fam]["FETCH_SIZE"] + by[fam]["WRITE_SIZE"]
    tot += b
    t = dur.get(fam, 0.0)
    out["families"][fam] = {"hbm_gb": round(b / 1e9, 3), "read_gb": round(2 * by[fam]["FETCH_SIZE"] / 1e9, 3),
                            "write_gb": round(by[fam]["WRITE_SIZE"] / 1e9, 3), "time_ms": round(t * 1e3, 3),
                            "gb_per_s": round(b / t / 1e9, 1) if t else None}
out["update_hbm_gb"] = round(tot / 1e9, 3)
out["update_window_s"] = round(span, 4)
out["kernel_time_s"] = round(sum(dur.values()), 4)
out["avg_tb_per_s_over_window"] = round(tot / span / 1e12, 3)
print(json.dumps(out, indent=1))
json.dump(out, open(os.path.join(root, "update_traffic.json"), "w"), indent=1)

"""Per-kernel averages of the PMC passes under a directory (scripts/pmc_kernels.sh)."""
import csv
import glob
import os
import sys
from collections import defaultdict

root = sys.argv[1]
vals = defaultdict(lambda: defaultdict(list))
for fn in sorted(glob.glob(os.path.join(root, "p*", "*counter_collection.csv"))):
    for row in csv.DictReader(open(fn)):
        kn = row["Kernel_Name"].replace("(anonymous namespace)::", "")
        name = kn.split("(")[0][-70:] + " grid=" + row["Grid_Size"]
        vals[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
for name, cs in sorted(vals.items()):
    avg = {k: sum(v) / len(v) for k, v in cs.items()}
    print(name)
    line = "   " + "  ".join(f"{k}={v:.4g}" for k, v in sorted(avg.items()))
    print(line)
    if "SQ_WAVE_CYCLES" in avg:
        wc = avg["SQ_WAVE_CYCLES"]
        print(f"   wait_any {avg.get('SQ_WAIT_ANY', 0) / wc:.2f}  active {avg.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f}")
    if "FETCH_SIZE" in avg:
        print(f"   fetch(x2) {2 * avg['FETCH_SIZE'] / 1024:.1f} MB  write {avg.get('WRITE_SIZE', 0) / 1024:.1f} MB")

"""Print the top kernels of a rocprofv3 *_kernel_stats.csv (name, calls, total ms, avg us, %)."""
import csv
import sys

fn = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rows = list(csv.DictReader(open(fn)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot / 1e6:.1f} ms")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
    t = float(r["TotalDurationNs"])
    print(f"{t / 1e6:9.2f} ms {100 * t / tot:5.1f}% n={int(r['Calls']):6d} avg {float(r['AverageNs']) / 1e3:8.2f} us  "
          f"{r['Name'][:100]}")

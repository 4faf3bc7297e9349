"""GPU busy fraction per idle-separated segment of a rocprofv3 kernel trace (union of kernel intervals
over all streams vs wall time): a low fraction with many short kernels means the host launch path,
not the GPU, sets the pace."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
gap = float(sys.argv[2]) if len(sys.argv) > 2 else 20e6
segs, cur = [], [rows[0]]
for a, b in zip(rows, rows[1:]):
    if int(b["Start_Timestamp"]) - max(int(r["End_Timestamp"]) for r in cur[-8:]) > gap:
        segs.append(cur)
        cur = []
    cur.append(b)
segs.append(cur)
for s in segs:
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in s)
    u, cs, ce = 0, iv[0][0], iv[0][1]
    for a, b in iv[1:]:
        if a > ce:
            u += ce - cs
            cs, ce = a, b
        else:
            ce = max(ce, b)
    u += ce - cs
    wall = iv[-1][1] - iv[0][0]
    print(f"{len(s):6d} kernels  wall {wall / 1e6:8.2f} ms  busy {u / 1e6:8.2f} ms ({100 * u / max(wall, 1):.0f}%)  "
          f"sum {sum(b - a for a, b in iv) / 1e6:8.2f} ms")

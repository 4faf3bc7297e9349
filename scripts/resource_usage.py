"""Print VGPR/SGPR/scratch/occupancy per kernel from hipcc -Rpass-analysis=kernel-resource-usage."""
import re
import subprocess
import sys

src = sys.argv[1]
out = subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-Iinclude", "-c", src,
                      "-Rpass-analysis=kernel-resource-usage", "-o", "/tmp/_ru.o"], capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"remark:\s+(.*?) \[-Rpass", line)
    if not m:
        continue
    body = m.group(1).strip()
    if body.startswith("Function Name:"):
        cur = body.split(":", 1)[1].strip()
        rows[cur] = {}
    elif cur and ":" in body:
        k, v = body.split(":", 1)
        rows[cur][k.strip()] = v.strip()
filt = sys.argv[2] if len(sys.argv) > 2 else ""
for name, r in rows.items():
    if filt in name:
        print(f"{name[:90]:90s} vgpr={r.get('VGPRs')} agpr={r.get('AGPRs')} sgpr={r.get('TotalSGPRs')} "
              f"scratch={r.get('ScratchSize [bytes/lane]')} occ={r.get('Occupancy [waves/SIMD]')} lds={r.get('LDS Size [bytes/block]')}")

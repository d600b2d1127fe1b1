#!/usr/bin/env python3
"""Per-kernel resource usage (VGPRs, spills, scratch, occupancy, LDS) of one HIP source for gfx950.

usage: python tools/kres.py csrc/ba_solver.hip [regex] [-D...]   (run from sfm-mvs-pipeline_amd/)
"""
import re
import subprocess
import sys

src = sys.argv[1]
pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 and not sys.argv[2].startswith("-D") else None
defs = [a for a in sys.argv[2:] if a.startswith("-D")]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "--offload-device-only",
       "-Rpass-analysis=kernel-resource-usage", "-c", src, "-o", "/dev/null"] + defs
out = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark: +(.*?): (.*?) \[-Rpass", line)
    if not m:
        continue
    key, val = m.group(1).strip(), m.group(2).strip()
    if key == "Function Name":
        dem = subprocess.run(["c++filt", val], capture_output=True, text=True).stdout.strip()
        cur = {"name": re.sub(r"\(.*", "", dem)}
        rows.append(cur)
    elif cur is not None:
        cur[key] = val
for r in rows:
    if pat and not pat.search(r["name"]):
        continue
    print(f"{r['name'][:60]:60s} vgpr {r.get('VGPRs', '?'):>4} agpr {r.get('AGPRs', '?'):>4} "
          f"spill {r.get('VGPRs Spill', '?'):>4} scratch {r.get('ScratchSize [bytes/lane]', '?'):>4} "
          f"occ {r.get('Occupancy [waves/SIMD]', '?'):>2} lds {r.get('LDS Size [bytes/block]', '?')}")

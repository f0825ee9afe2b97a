#!/usr/bin/env python3
"""Per-kernel register / spill / LDS report from hipcc -Rpass-analysis=kernel-resource-usage (dev tool).
    python tools/resources.py xhy-flash-attention_amd/csrc/fa_fwd.hip [--all]"""
import re
import subprocess
import sys

src = sys.argv[1]
out = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-x", "hip",
                      "-c", src, "-o", "/tmp/_res.o", "-Rpass-analysis=kernel-resource-usage"] + [a for a in sys.argv[2:] if a.startswith("-f") or a.startswith("-D")],
                     capture_output=True, text=True).stderr
cur, rows = None, []
for line in out.splitlines():
    m = re.search(r"remark: (?:\s*)(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|VGPRs Spill|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\S+)", line)
    if not m:
        continue
    k, v = m.group(1), m.group(2)
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k.split(" ")[0] + ("Spill" if "Spill" in k else "")] = v
for r in rows:
    bad = r.get("ScratchSize", "0") != "0" or r.get("VGPRsSpill", "0") != "0"
    if bad or "--all" in sys.argv:
        print(("SPILL " if bad else "      ") + r["name"], {k: v for k, v in r.items() if k != "name"})
print(f"{len(rows)} kernels, {sum(1 for r in rows if r.get('ScratchSize', '0') != '0' or r.get('VGPRsSpill', '0') != '0')} with scratch/spills")

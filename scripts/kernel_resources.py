#!/usr/bin/env python3
"""Print VGPR / SGPR / LDS / occupancy per kernel of a HIP source (hipcc -Rpass-analysis=kernel-resource-usage)."""
import re
import subprocess
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "orleans_amd/csrc/route_kernels.hip"
flt = sys.argv[2] if len(sys.argv) > 2 else ""
import os
if src.endswith(".log"):  # the remarks of a build already made (make lab DEFS="... -Rpass-analysis=kernel-resource-usage")
    class _R:
        stderr = open(src).read()
    r = _R()
else:
    r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-c", "-o", "/tmp/_kr.o", src,
                        "-Rpass-analysis=kernel-resource-usage"] + os.environ.get("DEFS", "").split(), capture_output=True,
                       text=True)
cur = None
rows = []
for line in r.stderr.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    t = m.group(1).strip()
    if t.startswith("Function Name:"):
        cur = {"name": subprocess.run(["c++filt"], input=t.split(":", 1)[1].strip(), capture_output=True,
                                      text=True).stdout.strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
for c in rows:
    n = re.sub(r"\(anonymous namespace\)::|orl::|void ", "", c["name"]).split("(")[0]
    if flt in n:
        print(f"{n:40s} VGPR={c.get('VGPRs'):>4} SGPR={c.get('TotalSGPRs'):>4} spill={c.get('VGPRs Spill')} LDS={c.get('LDS Size [bytes/block]'):>6} "
              f"waves/SIMD={c.get('Occupancy [waves/SIMD]')}")

#!/usr/bin/env python3
"""One step of a rocprofv3 kernel trace as a timeline (duration and the idle gap before each kernel).

    python scripts/ktimeline.py <dir-with-trace> [first-kernel-substring] [occurrence-from-end]

Finds the given occurrence (default 3rd from the end) of the first kernel of a step and prints the kernels up to the
next occurrence: the per-step launch chain of a small-batch workload (config 5), where gaps between dependent
kernels are the cost to cut."""
import csv
import glob
import sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
first = sys.argv[2] if len(sys.argv) > 2 else "k_scan_lb"
occ = int(sys.argv[3]) if len(sys.argv) > 3 else 3
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
a, b = idx[-occ], idx[-occ + 1] if occ > 1 else len(rows)
t0 = int(rows[a]["Start_Timestamp"])
prev_end = None
busy = 0
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").replace("orl::", "")
    gap = (s - prev_end) / 1e3 if prev_end is not None else 0.0
    busy += e - s
    print(f"{(s - t0) / 1e3:8.1f} us  +{gap:5.1f} gap  {(e - s) / 1e3:7.1f} us  {name[:90]}")
    prev_end = e
end = int(rows[b]["Start_Timestamp"]) if b < len(rows) else prev_end
print(f"step span {(end - t0) / 1e3:.1f} us, kernels busy {busy / 1e3:.1f} us, {b - a} kernels")

#!/usr/bin/env python3
"""Busy time per kernel over the last steps of a rocprofv3 kernel trace.

    python scripts/trace_sum.py <dir-with-trace> <marker-kernel-substring> <marker-launches-in-window> [steps]

The window starts at the N-th launch of the marker kernel counted from the end (e.g. 2 steps x 8 ranks x 4 chunks = 64
k_part_lb launches) and runs to the end of the trace.  Prints per-kernel busy microseconds per step, the span and the
busy total, so the GPU work of a multi-kernel step (the node rehearsal) can be attributed."""
import collections
import csv
import glob
import sys

marker, nwin = sys.argv[2], int(sys.argv[3])
steps = int(sys.argv[4]) if len(sys.argv) > 4 else 1
csvs = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)
if csvs:
    rows = list(csv.DictReader(open(csvs[0])))
else:  # rocprofv3's default rocpd output: the `kernels` view of the SQLite file
    import sqlite3
    db = sqlite3.connect(glob.glob(f"{sys.argv[1]}/**/*.db", recursive=True)[0])
    rows = [{"Kernel_Name": n, "Start_Timestamp": s, "End_Timestamp": e}
            for n, s, e in db.execute("select name, start, end from kernels")]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
a = idx[-nwin]
busy, cnt = collections.Counter(), collections.Counter()
for r in rows[a:]:
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").replace("orl::", "")
    name = name.split("(")[0][:60]
    busy[name] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    cnt[name] += 1
span = int(rows[-1]["End_Timestamp"]) - int(rows[a]["Start_Timestamp"])
tot = sum(busy.values())
print(f"window: {len(rows) - a} launches, span {span / 1e3 / steps:.1f} us/step, busy {tot / 1e3 / steps:.1f} us/step")
for k, v in busy.most_common():
    print(f"{v / 1e3 / steps:9.1f} us/step  {cnt[k] / steps:6.1f} launches/step  {v / cnt[k] / 1e3:8.1f} us avg  {k}")

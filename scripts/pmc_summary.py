#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs (one directory per pass) into per-kernel averages per dispatch.

Usage: python scripts/pmc_summary.py gpurun_out/prof [--json out.json] [--by-grid]
--by-grid keys the averages by (kernel, grid size): one kernel launched on different batch sizes (rank_cost_lab).
FETCH_SIZE/WRITE_SIZE are in KiB (rocprofv3 derived counters).  Per MI355X_MICROARCH.md §HBM, FETCH_SIZE reads
1/2 of the bytes of a wide coalesced stream on gfx950; the JSON reports both the raw value and TCC_EA0_RDREQ x 128 B.
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def kname(s):
    s = s.replace("(anonymous namespace)::", "")
    s = re.sub(r"^void ", "", s)
    return s.split("(")[0]


def main():
    root = sys.argv[1]
    agg = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(root, "pmc*", "pmc_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            k = kname(r["Kernel_Name"]) + (f" grid={r['Grid_Size']}" if "--by-grid" in sys.argv else "")
            agg[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
    out = collections.defaultdict(dict)
    for (k, c), v in sorted(agg.items()):
        out[k][c] = sum(v) / len(v)
        print(f"{k:60s} {c:24s} n={len(v):3d} avg={sum(v) / len(v):,.1f}")
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()

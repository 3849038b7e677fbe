#!/usr/bin/env python3
"""Join tools/probe_ceiling's timings with its two PMC passes into one table (profiles/r02_probe_ceiling.txt).

    python scripts/probe_ceiling_table.py gpurun_out/probe_ceiling.txt gpurun_out/pc_pmc1 gpurun_out/pc_pmc2

Dispatch order of tools/probe_ceiling: 2 fills, then per measured line 1 warm-up + 10 timed launches (counters averaged
over the 10).  FETCH_SIZE is in KiB and tallies every L2->memory-side read request at 64 B (MI355X_MICROARCH.md, HBM
section; profiles/r01_pmc_calibration.txt), so for random probes it counts fills, for the streamed headers half of the
bytes (128-B requests) — reported as tallied, per item.
"""
import csv
import glob
import sys
from collections import defaultdict


def counters(d):
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
    per = defaultdict(dict)
    for r in csv.DictReader(open(f)):
        per[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    return [per[k] for k in sorted(per)]


def main():
    lines = [l.rstrip() for l in open(sys.argv[1]) if " ms " in l]
    c = counters(sys.argv[2])
    f = counters(sys.argv[3])
    n = 64 << 20
    print(f"{'pattern':44s} {'ms':>7s} {'G/s':>7s} {'L2 hit':>7s} {'fetch B/item':>12s}")
    for i, l in enumerate(lines):
        name, rest = l[:44].strip(), l[44:].split()
        lo = 2 + 11 * i + 1
        reps = range(lo, lo + 10)
        hit = sum(c[k].get("TCC_HIT_sum", 0) for k in reps) / 10
        miss = sum(c[k].get("TCC_MISS_sum", 0) for k in reps) / 10
        fetch = sum(f[k].get("FETCH_SIZE", 0) for k in reps) / 10 * 1024
        print(f"{name:44s} {float(rest[0]):7.3f} {float(rest[2]):7.2f} {hit / max(hit + miss, 1):7.1%} {fetch / n:12.1f}")


if __name__ == "__main__":
    main()

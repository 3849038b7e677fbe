#!/usr/bin/env python3
"""Print a rocprofv3 kernel_stats.csv as a short table: python scripts/kstats.py <dir-with-trace>"""
import csv
import glob
import sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    name = r["Name"].replace("(anonymous namespace)::", "").replace("void ", "").replace("orl::", "")
    print(f"{name[:70]:70s} {r['Calls']:>5} {float(r['AverageNs']) / 1e3:9.1f} us {float(r['Percentage']):6.2f}%")

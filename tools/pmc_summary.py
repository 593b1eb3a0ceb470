#!/usr/bin/env python3
"""Summarise rocprofv3 kernel stats + PMC passes for one kernel (mean per dispatch)."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else "k_render"
for f in glob.glob(os.path.join(d, "trace", "*kernel_stats.csv")):
    for r in csv.DictReader(open(f)):
        if pat in r["Name"]:
            print(f"{r['Name'][:60]:60s} calls {r['Calls']:>4} avg {float(r['AverageNs'])/1e3:9.1f} us  min {float(r['MinNs'])/1e3:9.1f} us")
vals = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, "pmc*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        if pat in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(vals.items()):
    print(f"{k:32s} {sum(v)/len(v):16.4g}")

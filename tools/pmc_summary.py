#!/usr/bin/env python3
"""Diagnostic: per-kernel means of every counter in the rocprofv3 --pmc passes under a
directory (each pass a run of its own: <dir>/pmc*/.../*counter_collection.csv), with the
dispatch duration and the derived ratios used to read a latency-bound kernel:
  clock   GRBM_GUI_ACTIVE / 8 XCDs / duration (MI355X_MICROARCH.md "DVFS give-back")
  life    SQ_WAVE_CYCLES / SQ_WAVES (mean wave lifetime, counter units)
  wait    SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES, SQ_WAIT_ANY / SQ_WAVE_CYCLES
usage: pmc_summary.py DIR [kernel_substring ...]"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
want = sys.argv[2:]
for f in glob.glob(os.path.join(d, "trace", "*kernel_stats.csv")):  # tools/pmc_*.sh trace pass
    for r in csv.DictReader(open(f)):
        if not want or any(w in r["Name"] for w in want):
            print(f"{r['Name'][:60]:60s} calls {r['Calls']:>4} avg {float(r['AverageNs'])/1e3:9.1f} us  "
                  f"min {float(r['MinNs'])/1e3:9.1f} us")
vals = collections.defaultdict(lambda: collections.defaultdict(list))
durs = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, "pmc*", "**", "*counter_collection.csv"), recursive=True)):
    seen = set()
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0][:48]
        if want and not any(w in name for w in want):
            continue
        vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
        key = (f, r.get("Dispatch_Id"))
        if key not in seen and r.get("Start_Timestamp") and r.get("End_Timestamp"):
            seen.add(key)
            durs[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)


def mean(x):
    return sum(x) / len(x) if x else None


for name, c in sorted(vals.items(), key=lambda kv: -(mean(durs[kv[0]]) or 0) * len(durs[kv[0]])):
    m = {k: mean(v) for k, v in c.items()}
    du = mean(durs[name])
    out = [f"{name:48s} n={len(durs[name]):4d} dur={du:8.2f}us" if du else f"{name:48s}"]
    if m.get("GRBM_GUI_ACTIVE") and du:
        out.append(f"clock={m['GRBM_GUI_ACTIVE'] / 8 / (du * 1e3):.2f}GHz")
    if m.get("SQ_WAVES") and m.get("SQ_WAVE_CYCLES"):
        out.append(f"life={m['SQ_WAVE_CYCLES'] / m['SQ_WAVES']:.0f}")
    for k in ("SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_BUSY_CYCLES"):
        if m.get(k) is not None and m.get("SQ_WAVE_CYCLES"):
            out.append(f"{k[3:].lower()}/wc={m[k] / m['SQ_WAVE_CYCLES']:.2f}")
    print("  ".join(out))
    print("      " + "  ".join(f"{k}={v:.4g}" for k, v in sorted(m.items())))

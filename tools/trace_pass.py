#!/usr/bin/env python3
"""Diagnostic: per-kernel durations and inter-kernel gaps of the last encoder pass in a
rocprofv3 --kernel-trace database (rocpd sqlite), e.g. from tools/vit_prof.sh.
usage: trace_pass.py run_results.db|run_kernel_trace.csv [first_kernel_substring]"""
import sqlite3
import sys

if sys.argv[1].endswith(".csv"):  # rocprofv3 --output-format csv kernel trace
    import csv
    rows = sorted(((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                    int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"]))
                   for r in csv.DictReader(open(sys.argv[1]))), key=lambda r: r[1])
else:
    c = sqlite3.connect(sys.argv[1])
    rows = list(c.execute("select name, start, end, grid_x, workgroup_x from kernels order by start"))
first = sys.argv[2] if len(sys.argv) > 2 else "k_patchify"
starts = [i for i, r in enumerate(rows) if first in r[0]]
a = starts[-2] if len(starts) > 1 else starts[-1]
b = starts[-1] if len(starts) > 1 else len(rows)
seg = rows[a:b]
t0 = seg[0][1]
tot_k = 0
agg = {}
for i, (n, s, e, gx, wx) in enumerate(seg):
    gap = (s - seg[i - 1][2]) / 1e3 if i else 0.0
    d = (e - s) / 1e3
    tot_k += d
    short = n.split("(")[0][:60]
    agg.setdefault(short, [0, 0.0, 0.0])
    agg[short][0] += 1
    agg[short][1] += d
    agg[short][2] += gap
print(f"pass: {len(seg)} kernels, wall {(seg[-1][2] - t0) / 1e3:.1f} us, kernel sum {tot_k:.1f} us")
for k, (cnt, d, g) in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"{k:60s} x{cnt:3d}  {d:8.1f} us  avg {d / cnt:6.2f}  gaps before {g:7.1f} us")
if "--list" in sys.argv:  # every launch of the pass in order: duration, gap before, grid
    for i, (n, s, e, gx, wx) in enumerate(seg):
        gap = (s - seg[i - 1][2]) / 1e3 if i else 0.0
        print(f"{i:3d} {n.split('(')[0][:58]:58s} {(e - s) / 1e3:7.2f} us  gap {gap:6.2f}  grid {gx // max(wx, 1)} x {wx}")

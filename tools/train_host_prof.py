#!/usr/bin/env python3
"""Diagnostic: host (Python) time per training step by function -- cProfile over
bench.py --config train with many steps; prints the functions called about once or more per
step, by internal time per step."""
import cProfile
import pstats
import sys

sys.argv = ["bench.py", "--config", "train", "--steps", "300", "--warmup", "5"]
sys.path.insert(0, ".")
import bench  # noqa: E402

pr = cProfile.Profile()
pr.enable()
try:
    bench.main()
finally:
    pr.disable()
st = pstats.Stats(pr)
rows = []
for (fn, ln, name), (cc, nc, tt, ct, _) in st.stats.items():
    if nc >= 300:
        rows.append((tt / 305 * 1e6, ct / 305 * 1e6, nc / 305, f"{fn.split('/')[-1]}:{ln}({name})"))
rows.sort(reverse=True)
print("us/step tottime  cumtime  calls/step  function")
for tt, ct, n, f in rows[:45]:
    print(f"{tt:8.1f} {ct:8.1f} {n:6.1f}  {f}")

#!/bin/bash
# Round-4 GPU session 25: kernel durations of the ViT-S/16 and DINOv2-B/14 passes with the
# LayerNorm tail on / off (rocprofv3 kernel stats).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/r4s25
mkdir -p $O
for v in 1 0; do
  SCENEDINO_AMD_LN_TAIL=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/t$v -o run --output-format csv -- python3 bench.py --config vit --models vit-s16,dinov2-b14 --steps 5 --warmup 2 > $O/t$v.log 2>&1 || { tail -20 $O/t$v.log; exit 3; }
  python3 - <<PY
import csv
rows=list(csv.DictReader(open("$O/t$v/run_kernel_stats.csv")))
for r in rows[:14]: print("tail=$v", r["Name"][:60], r["Calls"], round(float(r["AverageNs"])/1e3,2))
PY
done
echo r4s25-done

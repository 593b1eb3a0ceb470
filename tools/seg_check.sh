#!/bin/bash
# Seg head: its GPU tests, the C5 bench (bf16 + fp8) and a kernel-trace profile of C5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/seg
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_seg.py tests/test_ssc.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 2; }
tail -2 $O/pytest.log
timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline > $O/c5.log 2>&1 || { tail -20 $O/c5.log; exit 3; }
timeout -k 10 300 python bench.py --config c5 --precision fp8 --no-cpu-baseline > $O/c5_fp8.log 2>&1 || { tail -20 $O/c5_fp8.log; exit 4; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --config c5 --no-cpu-baseline --steps 10 --warmup 3 > $O/c5_prof.log 2>&1 || { tail -20 $O/c5_prof.log; exit 5; }
for f in $O/c5.log $O/c5_fp8.log; do grep '^{' $f | cut -c1-200; done
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/seg/prof/**/*kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:8]:
    print(r["Name"][:60], r["Calls"], r["AverageNs"], r["Percentage"])
PY

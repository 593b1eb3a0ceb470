#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/e2eprof
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/t -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 3; }
f=$(find $O/t -name "*kernel_stats.csv" | head -1)
cut -d, -f1-4 "$f" | head -30 | cut -c1-200

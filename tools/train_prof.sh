#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/trainprof
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/t -o run --output-format csv -- python3 bench.py --config train --steps 10 --warmup 3 > $O/t.log 2>&1 || { tail -20 $O/t.log; exit 3; }
f=$(find $O/t -name "*kernel_stats.csv" | head -1)
cut -d, -f1-5 "$f" | head -25

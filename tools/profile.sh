#!/bin/bash
# rocprofv3 kernel trace + stats of a short bench, then separate PMC passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
OUT=gpurun_out/prof_${TAG:-r1}
mkdir -p $OUT
BENCH="bench.py --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline ${BENCH_ARGS}"
if [ -n "$LIST" ]; then rocprofv3 -L > $OUT/counters.txt 2>&1 || true; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $BENCH > $OUT/trace.log 2>&1 || { tail -20 $OUT/trace.log; exit 5; }
tail -3 $OUT/trace.log
i=0
for pmc in ${PMCS}; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc ${pmc//,/ } -d $OUT/pmc$i -o run --output-format csv -- python3 $BENCH > $OUT/pmc$i.log 2>&1 || { tail -20 $OUT/pmc$i.log; exit 6; }
done
find $OUT -name "*stats.csv" | head

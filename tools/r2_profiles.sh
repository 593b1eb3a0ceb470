#!/bin/bash
# Round evidence for C2 at each render pose: rocprofv3 kernel stats of the bench command,
# then FETCH_SIZE and WRITE_SIZE in separate PMC passes (MI355X_MICROARCH.md HBM section),
# summarised to profiles/<TAG>_traffic_<pose>.json by tools/traffic_json.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
TAG=${TAG:-r2}
O=gpurun_out/$TAG
mkdir -p $O
t() { timeout -k 10 "$@"; }
for pose in identity offset; do
  B="bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-end-to-end --$pose-pose"
  t 300 rocprofv3 --kernel-trace --stats -d $O/$pose/trace -o run --output-format csv -- python3 $B > $O/$pose.trace.log 2>&1 || { tail -20 $O/$pose.trace.log; exit 5; }
  t 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/$pose/pmc1 -o run --output-format csv -- python3 $B > $O/$pose.pmc1.log 2>&1 || { tail -20 $O/$pose.pmc1.log; exit 6; }
  t 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/$pose/pmc2 -o run --output-format csv -- python3 $B > $O/$pose.pmc2.log 2>&1 || { tail -20 $O/$pose.pmc2.log; exit 6; }
  python3 tools/traffic_json.py $O/$pose $O/${TAG}_traffic_$pose.json > /dev/null
  cp $O/$pose/trace/*kernel_stats.csv $O/${TAG}_c2_${pose}_kernel_stats.csv
  grep '^{' $O/$pose.trace.log | tail -1 > $O/${TAG}_c2_${pose}_bench_profiled.json
done
echo profiles-done

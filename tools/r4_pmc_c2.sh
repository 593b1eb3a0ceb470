#!/bin/bash
# Round-4 C2 HBM traffic per render pose: FETCH_SIZE / WRITE_SIZE passes (separate runs) of
# the bench at one pose each, summarised by tools/traffic_json.py into profiles/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/r4pmc
mkdir -p $O
for pose in offset identity; do
  B="bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-end-to-end --$pose-pose"
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$pose -o run --output-format csv -- python3 $B > $O/$pose.log 2>&1 || { tail -20 $O/$pose.log; exit 2; }
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/$pose/pmc1 -o run --output-format csv -- python3 $B > $O/${pose}_1.log 2>&1 || { tail -20 $O/${pose}_1.log; exit 3; }
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/$pose/pmc2 -o run --output-format csv -- python3 $B > $O/${pose}_2.log 2>&1 || { tail -20 $O/${pose}_2.log; exit 4; }
  python3 tools/traffic_json.py $O/$pose $O/r4_traffic_$pose.json > /dev/null
done
echo pmc-done

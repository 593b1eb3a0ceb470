#!/bin/bash
# C5 evidence: FETCH_SIZE and WRITE_SIZE of the voxel-path kernels (separate PMC passes),
# summarised to gpurun_out/c5t/c5_traffic.json by tools/traffic_json.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/c5t
mkdir -p $O
B="bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline"
timeout -k 10 180 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmc1 -o run --output-format csv -- python3 $B > $O/pmc1.log 2>&1 || { tail -20 $O/pmc1.log; exit 2; }
timeout -k 10 180 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmc2 -o run --output-format csv -- python3 $B > $O/pmc2.log 2>&1 || { tail -20 $O/pmc2.log; exit 3; }
python3 tools/traffic_json.py $O $O/c5_traffic.json

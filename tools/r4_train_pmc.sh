#!/bin/bash
# Round-4 training-step traffic: FETCH_SIZE / WRITE_SIZE passes (separate runs) of
# bench.py --config train for the shipped build and a diagnostic build without the
# grid-gradient atomics (noatom: wrong gradients, traffic split only), summarised per kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/r4trainpmc
mkdir -p $O
B="bench.py --config train --steps 5 --warmup 2 --no-graph --no-cpu-baseline"
for v in main noatom; do
  lib=""; [ $v != main ] && lib=scenedino_amd/variants/$v.so
  export SDHIP_LIB=$lib
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/$v/pmc1 -o run --output-format csv -- python3 $B > $O/${v}_1.log 2>&1 || { tail -20 $O/${v}_1.log; exit 2; }
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/$v/pmc2 -o run --output-format csv -- python3 $B > $O/${v}_2.log 2>&1 || { tail -20 $O/${v}_2.log; exit 3; }
  python3 tools/traffic_json.py $O/$v $O/r4_train_traffic_$v.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('$v', {k: (round(v['fetch_size_bytes_raw']/1e6,1), round(v['write_size_bytes']/1e6,1)) for k,v in d['kernels'].items() if v['fetch_size_bytes_raw'] is not None})"
done
echo trainpmc-done

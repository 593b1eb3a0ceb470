#!/bin/bash
# Round-4 GPU session 10: DPT layer microbenchmarks (tools/dpt_ops_bench.py) of the conv-tile
# variants, interleaved: main (chunk-major K, ReLU in LDS), relufrag, tapmaj, k_gemm path.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/r4s10
mkdir -p $O
t() { timeout -k 10 "$@"; }
for rep in 1 2 3; do
  for v in main relufrag tapmaj kgemm; do
    lib=""; big=1
    [ $v = relufrag ] || [ $v = tapmaj ] && lib=scenedino_amd/variants/$v.so
    [ $v = kgemm ] && big=0
    SDHIP_LIB=$lib SD_CONV_BIG=$big t 120 python -u tools/dpt_ops_bench.py > $O/ops_$v$rep.log 2>&1 || { tail -20 $O/ops_$v$rep.log; exit 5; }
    echo "$v $(tail -1 $O/ops_$v$rep.log)"
  done
done
echo r4s10-done

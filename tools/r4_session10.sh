#!/bin/bash
# Round-4 GPU session 10: DPT layer microbenchmarks (tools/dpt_ops_bench.py) of the conv-tile
# variants, interleaved: main (halo tiles), bigb (im2col tiles of the same build), relufrag,
# tapmaj (earlier im2col builds), k_gemm path.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/r4s10
mkdir -p $O
t() { timeout -k 10 "$@"; }
for rep in 1 2 3; do
  for v in main bigb relufrag tapmaj kgemm; do
    lib=""; big=1
    [ $v = relufrag ] || [ $v = tapmaj ] && lib=scenedino_amd/variants/$v.so
    [ $v = kgemm ] && big=0
    [ $v = bigb ] && big=b
    SDHIP_LIB=$lib SD_CONV_BIG=$big t 120 python -u tools/dpt_ops_bench.py > $O/ops_$v$rep.log 2>&1 || { tail -20 $O/ops_$v$rep.log; exit 5; }
    echo "$v $(tail -1 $O/ops_$v$rep.log)"
  done
done
t 300 python -u -m pytest tests/test_dpt.py -m gpu -v --timeout 120 --timeout-method thread > $O/pytest_dpt.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" $O/pytest_dpt.log | tail -30; exit 3; }
grep -E "passed|failed" $O/pytest_dpt.log | tail -2
echo r4s10-done

#!/bin/bash
# (ST_COL16 was measured and reverted -- profiles/r6_tile/rec36_ab.txt; the script records how)
# Diagnostic A/B: 36-B sample records (ST_COL16=1: red / green as an f16 pair) vs the 40-B
# records (variant col32), one and two rays per wave at K = 64; the render parity file first
# under both ray counts.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/${TAG:-col}
mkdir -p $O
t() { timeout -k 10 "$@"; }
[ -n "$NOTEST" ] || t 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "^E |FAILED" $O/pytest.log | head -20; tail -2 $O/pytest.log; exit 2; }
tail -1 $O/pytest.log
[ -n "$NOTEST" ] || SDHIP_TILE_RPW=2 t 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest_rpw2.log 2>&1 || { grep -E "^E |FAILED" $O/pytest_rpw2.log | head -20; tail -2 $O/pytest_rpw2.log; exit 2; }
tail -1 $O/pytest_rpw2.log
B="bench.py --no-cpu-baseline --no-end-to-end"
for rep in 1 2; do
  t 300 python -u $B > $O/c2_main.$rep.log 2>&1 || { tail -20 $O/c2_main.$rep.log; exit 4; }
  SDHIP_LIB=scenedino_amd/variants/col32.so t 300 python -u $B > $O/c2_col32.$rep.log 2>&1 || { tail -20 $O/c2_col32.$rep.log; exit 4; }
  SDHIP_TILE_RPW=2 t 300 python -u $B > $O/c2_rpw2.$rep.log 2>&1 || { tail -20 $O/c2_rpw2.$rep.log; exit 4; }
  t 300 python -u $B --config c1 > $O/c1_main.$rep.log 2>&1 || { tail -20 $O/c1_main.$rep.log; exit 4; }
  SDHIP_LIB=scenedino_amd/variants/col32.so t 300 python -u $B --config c1 > $O/c1_col32.$rep.log 2>&1 || { tail -20 $O/c1_col32.$rep.log; exit 4; }
done

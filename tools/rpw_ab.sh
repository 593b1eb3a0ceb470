#!/bin/bash
# Diagnostic A/B: two rays per wave at K = 64 (SDHIP_TILE_RPW=2) against the shipped one ray
# per wave, interleaved C2 bench lines, then the render parity file under RPW = 2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/${TAG:-rpw}
mkdir -p $O
t() { timeout -k 10 "$@"; }
B="bench.py --no-cpu-baseline --no-end-to-end"
for rep in 1 2; do
  t 300 python -u $B > $O/c2_main.$rep.log 2>&1 || { tail -20 $O/c2_main.$rep.log; exit 4; }
  SDHIP_TILE_RPW=2 t 300 python -u $B > $O/c2_rpw2.$rep.log 2>&1 || { tail -20 $O/c2_rpw2.$rep.log; exit 4; }
done
SDHIP_TILE_RPW=2 t 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 200 --timeout-method thread ${PYK:+-k "$PYK"} > $O/pytest_rpw2.log 2>&1 || { grep -E "^E |FAILED" $O/pytest_rpw2.log | head -20; tail -2 $O/pytest_rpw2.log; exit 2; }
tail -1 $O/pytest_rpw2.log

#!/bin/bash
# (ST_PACK was measured and reverted -- profiles/r6_tile/rpw2_k64_ab.txt; the script records how)
# Diagnostic A/B: packed per-part staging of split groups (ST_PACK=1, shipped candidate) vs
# one part per restage (variant nopack), C2 and C1 interleaved, and two rays per wave at K = 64
# with packing; the render parity file first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/${TAG:-pack}
mkdir -p $O
t() { timeout -k 10 "$@"; }
t 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "^E |FAILED" $O/pytest.log | head -20; tail -2 $O/pytest.log; exit 2; }
tail -1 $O/pytest.log
B="bench.py --no-cpu-baseline --no-end-to-end"
for rep in 1 2; do
  t 300 python -u $B > $O/c2_main.$rep.log 2>&1 || { tail -20 $O/c2_main.$rep.log; exit 4; }
  SDHIP_LIB=scenedino_amd/variants/nopack.so t 300 python -u $B > $O/c2_nopack.$rep.log 2>&1 || { tail -20 $O/c2_nopack.$rep.log; exit 4; }
  SDHIP_LIB=scenedino_amd/variants/tileold.so t 300 python -u $B > $O/c2_old.$rep.log 2>&1 || { tail -20 $O/c2_old.$rep.log; exit 4; }
  SDHIP_TILE_RPW=2 t 300 python -u $B > $O/c2_rpw2.$rep.log 2>&1 || { tail -20 $O/c2_rpw2.$rep.log; exit 4; }
  t 300 python -u $B --config c1 > $O/c1_main.$rep.log 2>&1 || { tail -20 $O/c1_main.$rep.log; exit 4; }
  SDHIP_LIB=scenedino_amd/variants/nopack.so t 300 python -u $B --config c1 > $O/c1_nopack.$rep.log 2>&1 || { tail -20 $O/c1_nopack.$rep.log; exit 4; }
done
SDHIP_TILE_RPW=2 t 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest_rpw2.log 2>&1 || { grep -E "^E |FAILED" $O/pytest_rpw2.log | head -20; tail -2 $O/pytest_rpw2.log; exit 2; }
tail -1 $O/pytest_rpw2.log

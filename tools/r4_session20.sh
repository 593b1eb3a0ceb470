#!/bin/bash
# Round-4 GPU session 20: the intermediate-layer token grids written by fc2's residual
# epilogue -- parity (unit + encoder), ViT / encode passes with it and without
# (SCENEDINO_AMD_FC2_GRID=0), interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/r4s20
mkdir -p $O
t() { timeout -k 10 "$@"; }
t 400 python -u -m pytest tests/test_vit.py tests/test_encoder.py tests/test_dpt.py -m gpu -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" $O/pytest.log | tail -30; exit 3; }
grep -E "passed|failed" $O/pytest.log | tail -2
for rep in 1 2; do
  for v in 1 0; do
    for c in vit encode; do
      SCENEDINO_AMD_FC2_GRID=$v t 300 python -u bench.py --config $c --models vit-s16,dinov2-b14 > $O/${c}_$v$rep.log 2>&1 || { tail -20 $O/${c}_$v$rep.log; exit 5; }
      python3 -c "import json,sys; d=json.loads([l for l in open('$O/${c}_$v$rep.log') if l.startswith('{')][-1]); print('$c fc2grid=$v', {m: round(v['ms_per_pass'],4) for m,v in d['models'].items()})"
    done
  done
done
echo r4s20-done

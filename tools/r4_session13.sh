#!/bin/bash
# Round-4 GPU session 13: cross-workgroup split-K with batched slice reads -- parity, then
# ViT / encode passes at SD_SPLITK_WG = 0 (off), 256 (one tile per CU), 512, interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/r4s13
mkdir -p $O
t() { timeout -k 10 "$@"; }
t 300 python -u -m pytest tests/test_vit.py tests/test_dpt.py -m gpu -k "split or conv3x3" -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" $O/pytest.log | tail -30; exit 3; }
grep -E "passed|failed" $O/pytest.log | tail -2
for rep in 1 2; do
  for wg in 0 256 512; do
    export SD_SPLITK_WG=$wg
    for c in vit encode; do
      t 300 python -u bench.py --config $c > $O/${c}_$wg$rep.log 2>&1 || { tail -20 $O/${c}_$wg$rep.log; exit 5; }
      python3 -c "import json,sys; d=json.loads([l for l in open('$O/${c}_$wg$rep.log') if l.startswith('{')][-1]); print('$c $wg', {m: round(v['ms_per_pass'],4) for m,v in d['models'].items()})"
    done
  done
done
echo r4s13-done

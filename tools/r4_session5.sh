#!/bin/bash
# Round-4 GPU session 5: k_lngemm packed-f32 LayerNorm (parity + A/B against the previous
# build), split-K ring depth 4 / 6 / 8 A/B on the ViT and encode passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/r4s5
mkdir -p $O
t() { timeout -k 10 "$@"; }
t 300 python -u -m pytest tests/test_vit.py tests/test_dpt.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 3; }
grep -E "passed|failed" $O/pytest.log | tail -2
for rep in 1 2; do
for v in prelg main rs6 rs8; do
  lib=""; [ $v != main ] && lib=scenedino_amd/variants/$v.so
  for c in vit encode; do
    SDHIP_LIB=$lib t 300 python -u bench.py --config $c > $O/${c}_$v.log 2>&1 || { tail -20 $O/${c}_$v.log; exit 5; }
    python3 -c "import json,sys; d=json.loads([l for l in open('$O/${c}_$v.log') if l.startswith('{')][-1]); print('$c $v', {m: round(v['ms_per_pass'],4) for m,v in d['models'].items()})"
  done
done
done
echo r4s5-done

#!/bin/bash
# Round-4 GPU session 24: the residual GEMM's LayerNorm tail (sd_gemm_resid_ln) -- ViT /
# encoder parity, then bench vit / encode with SCENEDINO_AMD_LN_TAIL=1 / 0 interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/r4s24
mkdir -p $O
t() { timeout -k 10 "$@"; }
t 600 python -u -m pytest tests/test_vit.py tests/test_encoder.py tests/test_dpt.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAIL|Error|assert" $O/pytest.log | tail -30; exit 3; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for v in 1 0; do
    for c in vit encode; do
      SCENEDINO_AMD_LN_TAIL=$v t 300 python -u bench.py --config $c > $O/${c}_$v.$rep.log 2>&1 || { tail -20 $O/${c}_$v.$rep.log; exit 5; }
      python3 -c "import json; d=json.loads([l for l in open('$O/${c}_$v.$rep.log') if l.startswith('{')][-1]); print('$c tail=$v', {k: round(m['ms_per_pass'],4) for k,m in d['models'].items()})"
    done
  done
done
echo r4s24-done

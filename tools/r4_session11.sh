#!/bin/bash
# Round-4 GPU session 11: DPT parity on the shipped conv dispatch (halo tiles at 96x320,
# im2col tiles elsewhere, fragment ReLU, cheaper sub-pixel epilogue), layer timings, encode.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/r4s11
mkdir -p $O
t() { timeout -k 10 "$@"; }
t 300 python -u -m pytest tests/test_dpt.py tests/test_encoder.py -m gpu -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" $O/pytest.log | tail -30; exit 3; }
grep -E "passed|failed" $O/pytest.log | tail -2
for rep in 1 2; do
  t 120 python -u tools/dpt_ops_bench.py > $O/ops$rep.log 2>&1 || { tail -20 $O/ops$rep.log; exit 5; }
  tail -1 $O/ops$rep.log
  t 300 python -u bench.py --config encode > $O/encode$rep.log 2>&1 || { tail -20 $O/encode$rep.log; exit 5; }
  python3 -c "import json,sys; d=json.loads([l for l in open('$O/encode$rep.log') if l.startswith('{')][-1]); print('encode', {m: round(v['ms_per_pass'],4) for m,v in d['models'].items()})"
done
echo r4s11-done

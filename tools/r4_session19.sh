#!/bin/bash
# Round-4 GPU session 19: 4 x 2 wave grid for the 128 x 64 conv tiles (main) vs 2 x 4
# (wgm2): parity, layer timings and encode passes, interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/r4s19
mkdir -p $O
t() { timeout -k 10 "$@"; }
t 300 python -u -m pytest tests/test_dpt.py -m gpu -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" $O/pytest.log | tail -30; exit 3; }
grep -E "passed|failed" $O/pytest.log | tail -2
for rep in 1 2; do
  for v in main wgm2; do
    lib=""; [ $v != main ] && lib=scenedino_amd/variants/$v.so
    SDHIP_LIB=$lib t 120 python -u tools/dpt_ops_bench.py > $O/ops_$v$rep.log 2>&1 || { tail -20 $O/ops_$v$rep.log; exit 5; }
    echo "$v $(tail -1 $O/ops_$v$rep.log)"
    SDHIP_LIB=$lib t 300 python -u bench.py --config encode > $O/encode_$v$rep.log 2>&1 || { tail -20 $O/encode_$v$rep.log; exit 5; }
    python3 -c "import json,sys; d=json.loads([l for l in open('$O/encode_$v$rep.log') if l.startswith('{')][-1]); print('encode $v', {m: round(v['ms_per_pass'],4) for m,v in d['models'].items()})"
  done
done
echo r4s19-done

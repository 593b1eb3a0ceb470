#!/bin/bash
# Round-4 GPU session 21: k_render_tile with padded hidden-sum rows (hspad: no 8-way bank
# conflicts in the DINO head's reads) -- render parity on that build, C2 / C1 A/B vs main.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/r4s21
mkdir -p $O
t() { timeout -k 10 "$@"; }
SDHIP_LIB=scenedino_amd/variants/hspad.so t 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAIL|Error|assert" $O/pytest.log | tail -30; exit 3; }
tail -1 $O/pytest.log
t 400 python -u -m pytest tests/test_seg.py -m gpu -q --timeout 120 --timeout-method thread > $O/seg.log 2>&1 || { grep -E "FAIL|Error|assert" $O/seg.log | tail -30; exit 4; }
tail -1 $O/seg.log
for rep in 1 2; do
  for v in main hspad; do
    lib=""; [ $v != main ] && lib=scenedino_amd/variants/$v.so
    for c in c2 c1; do
      SDHIP_LIB=$lib t 300 python -u bench.py --config $c --no-cpu-baseline --no-end-to-end > $O/${c}_$v$rep.log 2>&1 || { tail -20 $O/${c}_$v$rep.log; exit 5; }
      python3 -c "import json; d=json.loads([l for l in open('$O/${c}_$v$rep.log') if l.startswith('{')][-1]); print('$c $v', round(d['ms_per_step'],4), {p: (round(v['ms_per_step'],4), round(v['render_kernel_ms'],4)) for p,v in d['poses'].items()})"
    done
  done
done
echo r4s21-done

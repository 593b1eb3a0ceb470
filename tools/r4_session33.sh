#!/bin/bash
# Round-4 GPU session 33: two-pass buffer stores in the conv residual epilogues (session 31 layout)
# issued before the first store -- ViT / encoder parity, then bench vit / encode vs the
# previous build (variants/prev.so), 2 interleaved reps, and a kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/r4s33
mkdir -p $O
t() { timeout -k 10 "$@"; }
t 600 python -u -m pytest tests/test_dpt.py tests/test_encoder.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAIL|Error|assert" $O/pytest.log | tail -30; exit 3; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for v in main prev; do
    lib=""; [ $v != main ] && lib=scenedino_amd/variants/$v.so
    for c in vit encode; do
      SDHIP_LIB=$lib t 300 python -u bench.py --config $c > $O/${c}_$v.$rep.log 2>&1 || { tail -20 $O/${c}_$v.$rep.log; exit 5; }
      python3 -c "import json; d=json.loads([l for l in open('$O/${c}_$v.$rep.log') if l.startswith('{')][-1]); print('$c $v', {k: round(m['ms_per_pass'],4) for k,m in d['models'].items()})"
    done
  done
done
t 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --config vit --models vit-s16,dinov2-b14 --steps 5 --warmup 2 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 6; }
python3 - <<PY
import csv
for r in list(csv.DictReader(open("$O/prof/run_kernel_stats.csv")))[:12]: print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"])/1e3,2))
PY
echo r4s33-done

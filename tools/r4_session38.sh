#!/bin/bash
# Round-4 GPU session 38: k_composite_bwd recurrences in registers (K <= 64), dL/dfeat loaded once
# -- composite + training parity, then bench train vs the previous build, 2 reps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/r4s38
mkdir -p $O
t() { timeout -k 10 "$@"; }
t 600 python -u -m pytest tests/test_train.py tests/test_gpu_parity.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAIL|Error|assert" $O/pytest.log | tail -30; exit 3; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for v in main prev; do
    lib=""; [ $v != main ] && lib=scenedino_amd/variants/$v.so
    SDHIP_LIB=$lib t 300 python -u bench.py --config train > $O/train_$v.$rep.log 2>&1 || { tail -20 $O/train_$v.$rep.log; exit 5; }
    python3 -c "import json; d=json.loads([l for l in open('$O/train_$v.$rep.log') if l.startswith('{')][-1]); print('train $v', round(d['ms_per_step'],4))"
  done
done
t 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --config train --steps 5 --warmup 2 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 6; }
python3 - <<PY
import csv
for r in list(csv.DictReader(open("$O/prof/run_kernel_stats.csv")))[:10]: print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"])/1e3,2))
PY
echo r4s38-done

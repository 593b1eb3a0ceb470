#!/bin/bash
# Fast GPU iteration: render parity tests + C2 bench at both poses (+ optional extra
# command in $EXTRA).  Every GPU step has its own time limit; stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/quick
mkdir -p $O
t() { timeout -k 10 "$@"; }
t 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 2; }
tail -2 $O/pytest.log
t 300 python bench.py --no-end-to-end --no-cpu-baseline ${BENCH_ARGS} > $O/bench.log 2>&1 || { cat $O/bench.log; exit 4; }
python - $O/bench.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print("value", d["value"], "ms", d["ms_per_step"], "poses", json.dumps(d.get("poses")), "roofline", json.dumps(d.get("roofline")))
PY
if [ -n "$EXTRA" ]; then eval "$EXTRA" || exit 5; fi
echo quick-done

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
for pose in "" "--offset-pose"; do
  t 200 python bench.py --no-end-to-end --no-cpu-baseline $pose ${BENCH_ARGS} > $O/bench$pose.log 2>&1 || { cat $O/bench$pose.log; exit 4; }
  grep -o '"ms_per_step": [0-9.]*\|"render_kernel_ms": [0-9.]*\|"project_kernel_ms": [0-9.]*' $O/bench$pose.log | tr '\n' ' '; echo " $pose"
done
if [ -n "$EXTRA" ]; then eval "$EXTRA" || exit 5; fi
echo quick-done

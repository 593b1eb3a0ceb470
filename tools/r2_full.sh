#!/bin/bash
# GPU session: the whole -m gpu suite, smoke(), then the default bench line.
# Every GPU step has its own time limit; stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/full
mkdir -p $O
t() { timeout -k 10 "$@"; }
t 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 2; }
tail -2 $O/pytest.log
t 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 3; }
tail -1 $O/smoke.log
t 300 python bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 4; }
grep '^{' $O/bench.log
echo full-done

#!/bin/bash
# GPU session: the whole -m gpu suite (one process), stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/tests
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread "$@" > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 2; }
tail -3 $O/pytest.log

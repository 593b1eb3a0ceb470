#!/bin/bash
# One GPU session: build check, GPU parity tests, smoke, short bench.  Every GPU step
# has its own time limit; the script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONDONTWRITEBYTECODE=1
echo "== rocminfo"; (rocminfo | grep -m2 gfx) || true
timeout -k 10 900 python -m pytest tests -m gpu -q -rf --timeout 300 > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -30 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 3; }
cat gpurun_out/smoke.log
timeout -k 10 600 python bench.py --steps ${BENCH_STEPS:-10} --warmup 3 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { cat gpurun_out/bench.log; exit 4; }
cat gpurun_out/bench.log
exit $rc

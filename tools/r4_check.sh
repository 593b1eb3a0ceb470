#!/bin/bash
# Round-4 GPU iteration: selected parity tests, then C2 bench A/B of the projection kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/r4
mkdir -p $O
t() { timeout -k 10 "$@"; }
t 400 python -u -m pytest ${PYTEST_X--x} -q --timeout 200 --timeout-method thread ${TESTS:-tests/test_gpu_parity.py} > $O/pytest.log 2>&1
rc=$?
# rc 1 = test failures only (no crash, no timeout): PYTEST_KEEPGOING=1 still runs the benches
if [ $rc -ne 0 ]; then tail -40 $O/pytest.log; if [ $rc -ne 1 ] || [ -z "$PYTEST_KEEPGOING" ]; then exit 2; fi; fi
tail -2 $O/pytest.log
for rep in $(seq ${REPS:-1}); do
for v in ${VARIANTS:-new old}; do
  unset SDHIP_PROJ_OLD SDHIP_LIB
  if [ $v = old ]; then export SDHIP_PROJ_OLD=1; fi
  if [ -f scenedino_amd/variants/$v.so ]; then export SDHIP_LIB=scenedino_amd/variants/$v.so; fi
  t 300 python -u bench.py --no-end-to-end --no-cpu-baseline --no-fp16-line ${BENCH_ARGS} > $O/bench_$v.log 2>&1 || { cat $O/bench_$v.log; exit 4; }
  python - $O/bench_$v.log $v <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[2], "ms", round(d["ms_per_step"], 4), "poses", {k: (round(v["ms_per_step"], 4), round(v["render_kernel_ms"], 4), round(v["project_kernel_ms"], 4)) for k, v in d["poses"].items()})
PY
done
done
echo r4-done

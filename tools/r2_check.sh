#!/bin/bash
# GPU session: parity + multi-rank tests, C2 bench (both poses), 2-rank gloo dry runs of
# C2 and C5.  Every GPU step has its own time limit; stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/r2check
mkdir -p $O
t() { timeout -k 10 "$@"; }
t 400 python -u -m pytest tests/test_gpu_parity.py tests/test_multi_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 2; }
tail -2 $O/pytest.log
t 300 python bench.py --no-end-to-end --no-cpu-baseline > $O/c2.log 2>&1 || { cat $O/c2.log; exit 3; }
grep '^{' $O/c2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2', d['n_gpus'], round(d['value']/1e6,1), 'Mrays/s', {k: round(v['ms_per_step'],3) for k,v in d['poses'].items()}, 'frac', round(d['roofline']['frac'],3))"
t 300 python bench.py --gpus 2 --dist-backend gloo --steps 5 --warmup 2 --no-end-to-end --no-cpu-baseline > $O/c2_dry2.log 2>&1 || { cat $O/c2_dry2.log; exit 4; }
grep '^{' $O/c2_dry2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2 dry', d['n_gpus'], d['config']['parallelism'], d['config'].get('gathered_maps'))"
t 300 python bench.py --config c5 --gpus 2 --dist-backend gloo --steps 3 --warmup 1 > $O/c5_dry2.log 2>&1 || { cat $O/c5_dry2.log; exit 5; }
grep '^{' $O/c5_dry2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 dry', d['n_gpus'], d['config']['parallelism'], round(d['value']/1e6,1), 'Mvox/s')"
echo r2check-done

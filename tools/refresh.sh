#!/bin/bash
# One GPU session refreshing the round's evidence: GPU tests, smoke, the default bench
# (C2) + its rocprofv3 kernel stats and PMC passes, the training bench + its stats and PMC
# passes.  Every GPU step has its own time limit; stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/refresh
mkdir -p $O
t() { timeout -k 10 "$@"; }
t 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 2; }
tail -2 $O/pytest_gpu.log
t 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 3; }
t 300 python bench.py > $O/bench_c2.log 2>&1 || { cat $O/bench_c2.log; exit 4; }
grep -v amdgpu.ids $O/bench_c2.log | cut -c1-600
t 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-end-to-end > $O/prof_c2.log 2>&1 || { tail -20 $O/prof_c2.log; exit 5; }
t 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/prof_c2/pmc1 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-end-to-end > $O/pmc_c2_1.log 2>&1 || { tail -20 $O/pmc_c2_1.log; exit 6; }
t 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/prof_c2/pmc2 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-end-to-end > $O/pmc_c2_2.log 2>&1 || { tail -20 $O/pmc_c2_2.log; exit 6; }
t 300 python bench.py --config train > $O/bench_train.log 2>&1 || { cat $O/bench_train.log; exit 7; }
grep -v amdgpu.ids $O/bench_train.log | cut -c1-400
t 300 rocprofv3 --kernel-trace --stats -d $O/prof_train -o run --output-format csv -- python3 bench.py --config train --steps 5 --warmup 2 > $O/prof_train.log 2>&1 || { tail -20 $O/prof_train.log; exit 8; }
t 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/prof_train/pmc1 -o run --output-format csv -- python3 bench.py --config train --steps 3 --warmup 1 > $O/pmc_t_1.log 2>&1 || { tail -20 $O/pmc_t_1.log; exit 9; }
t 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/prof_train/pmc2 -o run --output-format csv -- python3 bench.py --config train --steps 3 --warmup 1 > $O/pmc_t_2.log 2>&1 || { tail -20 $O/pmc_t_2.log; exit 9; }
echo refresh-done

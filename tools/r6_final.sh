#!/bin/bash
# Round-6 evidence on the GPU box.  PART=1: the whole -m gpu suite, smoke(), the default
# bench line (C2), its rocprofv3 kernel stats and the FETCH_SIZE / WRITE_SIZE passes.
# PART=2: the other bench configs.  Every GPU step has its own time limit; stops at the
# first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/${TAG:-r6f}
mkdir -p $O
t() { timeout -k 10 "$@"; }
if [ "${PART:-1}" = 1 ]; then
t 700 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 2; }
tail -1 $O/pytest_gpu.log
t 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 3; }
t 300 python bench.py > $O/bench_c2.log 2>&1 || { tail -20 $O/bench_c2.log; exit 4; }
grep '^{' $O/bench_c2.log | cut -c1-400
B="bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-end-to-end"
t 300 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- python3 $B > $O/prof_c2.log 2>&1 || { tail -20 $O/prof_c2.log; exit 5; }
for pose in offset identity; do
  t 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/traffic_$pose/pmc1 -o run --output-format csv -- python3 $B --$pose-pose > $O/pmc1_$pose.log 2>&1 || { tail -20 $O/pmc1_$pose.log; exit 6; }
  t 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/traffic_$pose/pmc2 -o run --output-format csv -- python3 $B --$pose-pose > $O/pmc2_$pose.log 2>&1 || { tail -20 $O/pmc2_$pose.log; exit 7; }
done
echo part1-done
else
for c in c1 c5 c4 encode vit train; do
  t 300 python bench.py --config $c > $O/bench_$c.log 2>&1 || { tail -20 $O/bench_$c.log; exit 8; }
  grep '^{' $O/bench_$c.log | cut -c1-300
done
t 300 python bench.py --config c5 --precision fp8 > $O/bench_c5_fp8.log 2>&1 || { tail -20 $O/bench_c5_fp8.log; exit 9; }
echo part2-done
fi

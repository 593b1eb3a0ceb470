#!/bin/bash
# Round-3 training evidence on the GPU box: host issue time per phase, kernel stats and PMC
# HBM traffic (FETCH_SIZE / WRITE_SIZE passes) of the training bench; every GPU step has its
# own time limit, stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/r3train
mkdir -p $O
t() { timeout -k 10 "$@"; }
SCENEDINO_AMD_HOST_PROFILE=1 t 200 python bench.py --config train --steps 30 --warmup 5 > $O/host.log 2>&1 || { tail -20 $O/host.log; exit 2; }
grep "host issue" $O/host.log
t 200 python bench.py --config train --steps 30 --warmup 5 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 3; }
grep '^{' $O/bench.log | cut -c1-300
t 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --config train --steps 5 --warmup 2 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 4; }
t 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/prof/pmc1 -o run --output-format csv -- python3 bench.py --config train --steps 3 --warmup 1 > $O/pmc1.log 2>&1 || { tail -20 $O/pmc1.log; exit 5; }
t 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/prof/pmc2 -o run --output-format csv -- python3 bench.py --config train --steps 3 --warmup 1 > $O/pmc2.log 2>&1 || { tail -20 $O/pmc2.log; exit 6; }
echo train-evidence-done

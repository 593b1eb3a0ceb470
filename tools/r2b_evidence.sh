#!/bin/bash
# Round-2 (second session) evidence: C2 pose profiles + PMC traffic (tools/r2_profiles.sh),
# the training step's kernel stats + traffic, and the bench lines of every config.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/r2b
mkdir -p $O
t() { timeout -k 10 "$@"; }
TAG=r2 bash tools/r2_profiles.sh > $O/c2prof.log 2>&1 || { tail -20 $O/c2prof.log; exit 2; }
echo c2-profiles
B="bench.py --config train --steps 10 --warmup 3"
t 300 rocprofv3 --kernel-trace --stats -d $O/train/trace -o run --output-format csv -- python3 $B > $O/train.trace.log 2>&1 || { tail -20 $O/train.trace.log; exit 3; }
t 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/train/pmc1 -o run --output-format csv -- python3 $B > $O/train.pmc1.log 2>&1 || { tail -20 $O/train.pmc1.log; exit 4; }
t 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/train/pmc2 -o run --output-format csv -- python3 $B > $O/train.pmc2.log 2>&1 || { tail -20 $O/train.pmc2.log; exit 4; }
python3 tools/traffic_json.py $O/train $O/r2_train_traffic.json > /dev/null
cp $O/train/trace/*kernel_stats.csv $O/r2_train_kernel_stats.csv
echo train-profiles
t 300 python bench.py > $O/bench_c2.log 2>&1 || { tail -20 $O/bench_c2.log; exit 5; }
t 300 python bench.py --config train > $O/bench_train.log 2>&1 || { tail -20 $O/bench_train.log; exit 6; }
t 300 python bench.py --config vit > $O/bench_vit.log 2>&1 || { tail -20 $O/bench_vit.log; exit 7; }
t 300 python bench.py --config encode > $O/bench_encode.log 2>&1 || { tail -20 $O/bench_encode.log; exit 8; }
t 300 python bench.py --config c5 > $O/bench_c5_bf16.log 2>&1 || { tail -20 $O/bench_c5_bf16.log; exit 9; }
t 300 python bench.py --config c5 --precision fp8 > $O/bench_c5_fp8.log 2>&1 || { tail -20 $O/bench_c5_fp8.log; exit 10; }
t 300 python bench.py --config c4 --no-cpu-baseline > $O/bench_c4.log 2>&1 || { tail -20 $O/bench_c4.log; exit 11; }
for f in $O/bench_*.log; do echo "== $f"; grep '^{' $f | cut -c1-250; done
echo evidence-done

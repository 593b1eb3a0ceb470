#!/bin/bash
# One parameterised GPU session (replaces the per-session scripts of rounds 2-4).
#
#   tools/gpu_session.sh TAG STEP [STEP ...]
#
# Steps (run in order; every GPU step under its own time limit; the session stops at the
# first failure, so nothing runs on the GPU after a fault, abort or timeout):
#   pytest[:ARGS]        python -m pytest -m gpu ARGS (default: the whole tests/ directory);
#                        ARGS uses ',' for spaces, e.g. pytest:tests/test_gpu_parity.py,-k,lowp
#   smoke                __graft_entry__.smoke()
#   bench:CFG[:ARGS]     python bench.py --config CFG ARGS (',' for spaces)
#   prof:CFG[:ARGS]      rocprofv3 --kernel-trace --stats of a short bench run
#   pmc:CFG:COUNTERS[:ARGS] one rocprofv3 --pmc pass (COUNTERS ',' separated, within one
#                        block's limit; ARGS: extra bench.py arguments, ',' for spaces)
#   env:VAR=VALUE        export VAR for the following steps (env:VAR= unsets it)
#   ab:CFG:VARIANT:REPS  interleaved bench runs of the shipped library and
#                        scenedino_amd/variants/VARIANT.so (tools/build_variant.py)
#   py:SCRIPT[:ARGS]     python SCRIPT ARGS (a GPU tool under tools/)
# Output: gpurun_out/TAG/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
t() { timeout -k 10 "$@"; }
summ() {  # kernel stats: name, calls, average us
  python3 - "$1" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:14]:
    print(f'{r["Name"][:72]:72s} {r["Calls"]:>6s} {float(r["AverageNs"])/1e3:9.2f} us')
PY
}
line() { grep '^{' "$1" | tail -1 | cut -c1-${2:-600}; }
n=0
for step in "$@"; do
  n=$((n + 1))
  IFS=':' read -r kind a1 a2 a3 <<< "$step"
  case $kind in
    pytest)
      args=${a1//,/ }; [ -z "$args" ] && args=tests
      t 900 python -u -m pytest $args -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest$n.log 2>&1 \
        || { grep -E "FAIL|Error|assert|Timeout" $O/pytest$n.log | tail -40; tail -5 $O/pytest$n.log; exit 2; }
      tail -1 $O/pytest$n.log ;;
    smoke)
      t 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 3; }
      tail -1 $O/smoke.log ;;
    bench)
      f=$O/bench_${a1}$n.log
      t 400 python -u bench.py --config $a1 ${a2//,/ } > $f 2>&1 || { tail -20 $f; exit 4; }
      line $f ;;
    prof)
      d=$O/prof_${a1}$n
      t 300 rocprofv3 --kernel-trace --stats -d $d -o run --output-format csv -- \
        python3 bench.py --config $a1 --steps 5 --warmup 2 --no-cpu-baseline --no-end-to-end ${a2//,/ } > $d.log 2>&1 \
        || { tail -20 $d.log; exit 5; }
      summ $d/run_kernel_stats.csv ;;
    pmc)
      d=$O/pmc_${a1}$n
      t 180 rocprofv3 --kernel-trace --pmc ${a2//,/ } -d $d -o run --output-format csv -- \
        python3 bench.py --config $a1 --steps 3 --warmup 1 --no-cpu-baseline --no-end-to-end ${a3//,/ } > $d.log 2>&1 \
        || { tail -20 $d.log; exit 6; }
      echo "pmc $a1 $a2 -> $d" ;;
    ab)
      for rep in $(seq 1 ${a3:-2}); do
        for v in main $a2; do
          lib=""; [ $v != main ] && lib=scenedino_amd/variants/$v.so
          f=$O/ab_${a1}_$v.$rep.log
          SDHIP_LIB=$lib t 300 python -u bench.py --config $a1 --no-cpu-baseline > $f 2>&1 || { tail -20 $f; exit 7; }
          python3 -c "import json,sys; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); print('ab $a1 $v', round(d['ms_per_step'],4))"
        done
      done ;;
    env)
      v=${step#env:}; if [ -z "${v#*=}" ]; then unset "${v%%=*}"; else export "$v"; fi
      echo "env $v" ;;
    py)
      f=$O/py$n.log
      t 400 python -u $a1 ${a2//,/ } > $f 2>&1 || { tail -30 $f; exit 8; }
      tail -40 $f ;;
    *) echo "unknown step $step"; exit 9 ;;
  esac
done
echo "$TAG done"

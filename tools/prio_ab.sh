#!/bin/bash
# Diagnostic A/B: k_render_tile static issue priority (ST_PRIO variants prio1 / prio2 vs the
# shipped build), C2 and C1 interleaved, 3 rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/${TAG:-prio}
mkdir -p $O
t() { timeout -k 10 "$@"; }
B="bench.py --no-cpu-baseline --no-end-to-end"
for rep in 1 2 3; do
  for v in main ${VARIANTS:-prio1 prio2}; do
    lib=""; [ $v != main ] && lib=scenedino_amd/variants/$v.so
    for c in c2 c1; do
      SDHIP_LIB=$lib t 300 python -u $B --config $c > $O/${c}_$v.$rep.log 2>&1 || { tail -20 $O/${c}_$v.$rep.log; exit 4; }
    done
  done
done

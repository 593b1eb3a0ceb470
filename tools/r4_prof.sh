#!/bin/bash
# Round-4 diagnostics: projection A/B, tile phase split, ViT kernel traces.  Every GPU step
# has its own time limit; the script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/r4p
mkdir -p $O
t() { timeout -k 10 "$@"; }
if [ -z "$SKIP_AB" ]; then
VARIANTS=${VARIANTS:-"new pjhalf"} REPS=${REPS:-2} TESTS=${TESTS:-tests/test_reconstruct.py} tools/r4_check.sh || exit 3
fi
if [ -z "$SKIP_TPROF" ]; then
SDHIP_LIB=scenedino_amd/variants/tprof.so t 200 python tools/tile_prof.py > $O/tile_prof_k64.txt 2>&1 || { cat $O/tile_prof_k64.txt; exit 4; }
cat $O/tile_prof_k64.txt
fi
if [ -z "$SKIP_VITOPS" ]; then
t 200 python tools/vit_ops_bench.py > $O/vit_ops.json 2>&1 || { cat $O/vit_ops.json; exit 6; }
tail -1 $O/vit_ops.json
fi
if [ -z "$SKIP_VIT" ]; then
for m in ${MODELS:-vit-s16 dinov2-b14}; do
  t 240 rocprofv3 --kernel-trace -d $O/vit_$m -o run -- python3 bench.py --config vit --models $m --steps 10 --warmup 3 > $O/vit_$m.log 2>&1 || { tail -20 $O/vit_$m.log; exit 5; }
  db=$(find $O/vit_$m -name "*.db" | head -1)
  python3 tools/trace_pass.py $db k_patchify --list > $O/vit_trace_$m.txt 2>&1 || true
  head -40 $O/vit_trace_$m.txt
done
fi
if [ -z "$SKIP_TRAIN" ]; then
for mode in graph eager; do
  extra=""; [ $mode = graph ] && extra="--graph"
  SCENEDINO_AMD_HOST_PROFILE=1 t 300 python -u bench.py --config train --steps 20 --warmup 3 $extra > $O/train_$mode.log 2>&1 || { tail -30 $O/train_$mode.log; exit 7; }
  python - $O/train_$mode.log $mode <<'PY'
import json, sys
lines = open(sys.argv[1]).read().splitlines()
d = json.loads([l for l in lines if l.startswith("{")][-1])
print(sys.argv[2], "ms/step", round(d["ms_per_step"], 4), d.get("step_issue"), [l for l in lines if l.startswith("host issue")])
PY
done
fi
echo r4p-done

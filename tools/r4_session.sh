#!/bin/bash
# Round-4 GPU session: parity tests of the shipped library, the same GEMM tests on the
# LDS-DMA ring variant, then A/B benches (projection, ViT ops, encode), the graphed
# training step and the tile phase split.  Every GPU step has its own time limit; a crash,
# abort or timeout ends the script (test failures alone do not, with KEEPGOING=1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/r4s
mkdir -p $O
t() { timeout -k 10 "$@"; }
pt() {  # name, then pytest args
  local n=$1; shift
  t 600 python -u -m pytest -q --timeout 200 --timeout-method thread "$@" > $O/pytest_$n.log 2>&1
  local rc=$?
  tail -3 $O/pytest_$n.log
  if [ $rc -ne 0 ]; then grep -E "^FAILED|^ERROR" $O/pytest_$n.log | head -20; fi
  if [ $rc -ne 0 ] && { [ $rc -ne 1 ] || [ -z "$KEEPGOING" ]; }; then exit 2; fi
}
pt main ${TESTS_MAIN:-tests/test_gpu_parity.py tests/test_vit.py tests/test_dpt.py tests/test_encoder.py tests/test_train.py tests/test_visualization.py}
if [ -f scenedino_amd/variants/ring.so ]; then
  SDHIP_LIB=scenedino_amd/variants/ring.so pt ring tests/test_vit.py tests/test_dpt.py tests/test_encoder.py
fi
bl() { python - "$@" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
k = sys.argv[2]
if "poses" in d:
    print(k, "ms", round(d["ms_per_step"], 4), {p: (round(v["ms_per_step"], 4), round(v["render_kernel_ms"], 4), round(v["project_kernel_ms"], 4)) for p, v in d["poses"].items()})
elif "models" in d:
    print(k, {m: round(v["ms_per_pass"], 4) for m, v in d["models"].items()})
else:
    print(k, "ms", round(d["ms_per_step"], 4), d.get("step_issue"))
PY
}
for rep in 1 2; do
  for v in main pjhalf; do
    lib=""; [ $v != main ] && lib=scenedino_amd/variants/$v.so
    SDHIP_LIB=$lib t 300 python -u bench.py --no-end-to-end --no-cpu-baseline --no-fp16-line > $O/c2_$v.log 2>&1 || { tail -20 $O/c2_$v.log; exit 4; }
    bl $O/c2_$v.log c2_$v
  done
done
for v in main ring; do
  lib=""; [ $v != main ] && lib=scenedino_amd/variants/$v.so
  SDHIP_LIB=$lib t 200 python tools/vit_ops_bench.py > $O/vitops_$v.json 2>&1 || { tail -20 $O/vitops_$v.json; exit 5; }
  tail -1 $O/vitops_$v.json
  SDHIP_LIB=$lib t 300 python -u bench.py --config encode > $O/encode_$v.log 2>&1 || { tail -20 $O/encode_$v.log; exit 5; }
  bl $O/encode_$v.log encode_$v
  SDHIP_LIB=$lib t 300 python -u bench.py --config vit > $O/vit_$v.log 2>&1 || { tail -20 $O/vit_$v.log; exit 5; }
  bl $O/vit_$v.log vit_$v
done
for mode in graph eager; do
  extra=""; [ $mode = graph ] && extra="--graph"
  SCENEDINO_AMD_HOST_PROFILE=1 t 300 python -u bench.py --config train --steps 20 --warmup 3 $extra > $O/train_$mode.log 2>&1 || { tail -30 $O/train_$mode.log; exit 7; }
  bl $O/train_$mode.log train_$mode; grep "host issue" $O/train_$mode.log
done
SDHIP_LIB=scenedino_amd/variants/tprof.so t 200 python tools/tile_prof.py > $O/tile_prof_k64.txt 2>&1 || { cat $O/tile_prof_k64.txt; exit 8; }
cat $O/tile_prof_k64.txt
echo r4s-done

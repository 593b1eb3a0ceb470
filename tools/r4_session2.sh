#!/bin/bash
# Round-4 GPU session 2: the driver's default bench line, ring-32 GEMM A/B (ViT and encode
# passes + per-kernel traces), the graphed training step, the tile phase split.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/r4s2
mkdir -p $O
t() { timeout -k 10 "$@"; }
bl() { python - "$@" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
k = sys.argv[2]
if "poses" in d:
    print(k, "ms", round(d["ms_per_step"], 4), {p: (round(v["ms_per_step"], 4), round(v["render_kernel_ms"], 4), round(v["project_kernel_ms"], 4)) for p, v in d["poses"].items()}, "fp16", (d.get("fp16_default") or {}).get("ms_per_step"), "e2e", (d.get("end_to_end") or {}).get("ms_per_frame"))
elif "models" in d:
    print(k, {m: round(v["ms_per_pass"], 4) for m, v in d["models"].items()})
else:
    print(k, "ms", round(d["ms_per_step"], 4), d.get("step_issue"))
PY
}
t 400 python -u bench.py > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 3; }
bl $O/bench_default.log default
for rep in 1 2; do
for v in main ring; do
  lib=""; [ $v != main ] && lib=scenedino_amd/variants/$v.so
  SDHIP_LIB=$lib t 300 python -u bench.py --config vit > $O/vit_$v.log 2>&1 || { tail -20 $O/vit_$v.log; exit 5; }
  bl $O/vit_$v.log vit_$v
  SDHIP_LIB=$lib t 300 python -u bench.py --config encode > $O/encode_$v.log 2>&1 || { tail -20 $O/encode_$v.log; exit 5; }
  bl $O/encode_$v.log encode_$v
done
done
for v in main ring; do
  lib=""; [ $v != main ] && lib=scenedino_amd/variants/$v.so
  SDHIP_LIB=$lib t 240 rocprofv3 --kernel-trace -d $O/enc_$v -o run -- python3 bench.py --config encode --models vit-s16 --steps 10 --warmup 3 > $O/enc_$v.log 2>&1 || { tail -20 $O/enc_$v.log; exit 6; }
  db=$(find $O/enc_$v -name "*.db" | head -1)
  python3 tools/trace_pass.py $db k_patchify > $O/enc_trace_$v.txt 2>&1; head -25 $O/enc_trace_$v.txt
done
for mode in graph eager; do
  extra=""; [ $mode = graph ] && extra="--graph"
  SCENEDINO_AMD_HOST_PROFILE=1 t 300 python -X faulthandler -u bench.py --config train --steps 20 --warmup 3 $extra > $O/train_$mode.log 2>&1 || { tail -40 $O/train_$mode.log; exit 7; }
  bl $O/train_$mode.log train_$mode; grep "host issue" $O/train_$mode.log
done
SDHIP_LIB=scenedino_amd/variants/tprof.so t 200 python tools/tile_prof.py > $O/tile_prof_k64.txt 2>&1 || { cat $O/tile_prof_k64.txt; exit 8; }
cat $O/tile_prof_k64.txt
echo r4s2-done

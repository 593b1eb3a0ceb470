#!/bin/bash
# Diagnostic: k_project time (C2 offset pose and C5) of the shipped library vs the variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in $(seq ${REPS:-2}); do
for lib in scenedino_amd/libsdhip.so $(ls scenedino_amd/variants/*.so 2>/dev/null); do
  n=$(basename $lib .so)
  SDHIP_LIB=$lib timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-end-to-end --offset-pose > gpurun_out/pab_$n.log 2>&1 || { tail -5 gpurun_out/pab_$n.log; exit 7; }
  SDHIP_LIB=$lib timeout -k 10 200 python bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/pab5_$n.log 2>&1 || { tail -5 gpurun_out/pab5_$n.log; exit 8; }
  python - "$n" <<'PY'
import json, sys
n = sys.argv[1]
d = json.loads([l for l in open(f"gpurun_out/pab_{n}.log") if l.startswith("{")][-1])
e = json.loads([l for l in open(f"gpurun_out/pab5_{n}.log") if l.startswith("{")][-1])
p = d["poses"]["offset"]
print(n, "c2 step", round(d["ms_per_step"], 4), "project", round(p["project_kernel_ms"], 4), "render", round(p["render_kernel_ms"], 4), "| c5 step", round(e["ms_per_step"], 4))
PY
done
done

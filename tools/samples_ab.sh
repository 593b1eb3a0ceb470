#!/bin/bash
# Diagnostic: C2 frame with and without the per-sample weight / alpha outputs (3 reps).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sab
for rep in 1 2 3; do for ns in 0 1; do
  SCENEDINO_AMD_BENCH_NO_SAMPLES=$ns timeout -k 10 200 python bench.py --no-cpu-baseline --no-end-to-end --offset-pose --steps 30 > gpurun_out/sab/$ns.$rep.log 2>&1 || { tail -20 gpurun_out/sab/$ns.$rep.log; exit 4; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/sab/$ns.$rep.log') if l.startswith('{')][0]); r=d['roofline']; print('no_samples=$ns', round(d['ms_per_step'],4), 'render', round(r['render_kernel_ms'],4))"
done; done

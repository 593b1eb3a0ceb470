#!/bin/bash
# Diagnostic: training step with the grid_sample backward fused into k_mlp_bwd (default)
# and unfused (SCENEDINO_AMD_FUSED_SCATTER=0: dX rows + k_field_gather_bwd), both render
# poses; prints ms per step and the backward kernel times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for pose in "" "--offset-pose"; do
  for f in 1 0; do
    n=train_f${f}${pose:+_offset}
    SCENEDINO_AMD_FUSED_SCATTER=$f timeout -k 10 200 python bench.py --config train --steps 30 --warmup 5 $pose > gpurun_out/$n.log 2>&1 || { tail -5 gpurun_out/$n.log; exit 7; }
    python -c "import json; d=json.loads([l for l in open('gpurun_out/$n.log') if l.startswith('{')][-1]); r=d['roofline']; print('$n', round(d['ms_per_step'],3), 'mlp_bwd', round(r['mlp_bwd_ms'],4), 'gather_bwd', round(r['gather_bwd_ms'],4), 'frac', r['frac'])"
  done
done

#!/bin/bash
# Round-4 GPU session 18: LayerNorm fused into the C = 768 qkv / fc1 GEMMs (DINOv2-B/14,
# SCENEDINO_AMD_LN_GEMM=all) vs the unfused default, ViT passes interleaved; the C2 line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/r4s18
mkdir -p $O
t() { timeout -k 10 "$@"; }
for rep in 1 2; do
  for v in 1 all; do
    SCENEDINO_AMD_LN_GEMM=$v t 300 python -u bench.py --config vit --models dinov2-b14,vit-s16 > $O/vit_$v$rep.log 2>&1 || { tail -20 $O/vit_$v$rep.log; exit 5; }
    python3 -c "import json,sys; d=json.loads([l for l in open('$O/vit_$v$rep.log') if l.startswith('{')][-1]); print('vit ln=$v', {m: round(v['ms_per_pass'],4) for m,v in d['models'].items()})"
  done
done
t 400 python -u bench.py --no-cpu-baseline --no-end-to-end > $O/c2.log 2>&1 || { tail -20 $O/c2.log; exit 6; }
python3 -c "import json; d=json.loads([l for l in open('$O/c2.log') if l.startswith('{')][-1]); print('c2', round(d['ms_per_step'],4), {p: round(v['ms_per_step'],4) for p,v in d['poses'].items()})"
echo r4s18-done

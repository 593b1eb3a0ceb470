#!/bin/bash
# Round-4 GPU session 27: does the LayerNorm-tail plumbing cost the default residual GEMM
# anything?  bench vit: shipped build vs -DVT_LN_TAIL=0 (tail branches compiled out), 2 reps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/r4s27
mkdir -p $O
for rep in 1 2; do
  for v in main notail; do
    lib=""; [ $v != main ] && lib=scenedino_amd/variants/$v.so
    SDHIP_LIB=$lib timeout -k 10 300 python -u bench.py --config vit > $O/vit_$v.$rep.log 2>&1 || { tail -20 $O/vit_$v.$rep.log; exit 5; }
    python3 -c "import json; d=json.loads([l for l in open('$O/vit_$v.$rep.log') if l.startswith('{')][-1]); print('vit $v', {k: round(m['ms_per_pass'],4) for k,m in d['models'].items()})"
  done
done
echo r4s27-done

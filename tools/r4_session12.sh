#!/bin/bash
# Round-4 GPU session 12: cross-workgroup split-K on the 32 x 32 tiles -- parity (GEMM, DPT,
# encoder), ViT / encode passes with it (default) and without (SD_SPLITK_WG=0), interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/r4s12
mkdir -p $O
t() { timeout -k 10 "$@"; }
for rep in 1 2; do
  for v in split nosplit; do
    if [ $v = nosplit ]; then export SD_SPLITK_WG=0; else export SD_SPLITK_WG=256; fi
    for c in vit encode; do
      t 300 python -u bench.py --config $c > $O/${c}_$v$rep.log 2>&1 || { tail -20 $O/${c}_$v$rep.log; exit 5; }
      python3 -c "import json,sys; d=json.loads([l for l in open('$O/${c}_$v$rep.log') if l.startswith('{')][-1]); print('$c $v', {m: round(v['ms_per_pass'],4) for m,v in d['models'].items()})"
    done
  done
done
export SD_SPLITK_WG=256
t 240 rocprofv3 --kernel-trace -d $O/enc -o run -- python3 bench.py --config encode --models vit-s16 --steps 10 --warmup 3 > $O/enc.log 2>&1 || { tail -20 $O/enc.log; exit 6; }
db=$(find $O/enc -name "*.db" | head -1)
python3 tools/trace_pass.py $db k_patchify --list > $O/enc_trace.txt 2>&1; head -30 $O/enc_trace.txt
echo r4s12-done

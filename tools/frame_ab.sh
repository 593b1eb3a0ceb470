#!/bin/bash
# A/B of the fused frame inputs (SCENEDINO_AMD_FRAME_FUSED=1, default) against their own
# launch (=0): interleaved bench runs of CFG (default c5), ms per step.
set -o pipefail
mkdir -p gpurun_out/frab
for rep in 1 2 3; do
  for v in 1 0; do
    f=gpurun_out/frab/${1:-c5}.$v.$rep.log
    SCENEDINO_AMD_FRAME_FUSED=$v timeout -k 10 300 python -u bench.py --config ${1:-c5} --no-cpu-baseline --no-end-to-end > $f 2>&1 || { tail -5 $f; exit 3; }
    python3 -c "import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); print('${1:-c5} fused=$v', round(d['ms_per_step'],4))"
  done
done

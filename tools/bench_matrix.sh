#!/bin/bash
# Short bench over precisions / poses (no CPU baseline), each step time-limited.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for prec in ${PRECS:-bf16 fp16 fp32}; do
  for extra in "" "--offset-pose"; do
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --precision $prec $extra > gpurun_out/bm_${prec}${extra}.log 2>&1 || { cat gpurun_out/bm_${prec}${extra}.log; exit 7; }
    python -c "import json,sys; d=json.loads(open('gpurun_out/bm_${prec}${extra}.log').read().strip().splitlines()[-1]); print('$prec','$extra', round(d['value']/1e6,2),'Mrays/s', round(d['ms_per_step'],3),'ms', 'kernel', round(d['roofline']['kernel_ms'],3),'ms frac', round(d['roofline']['frac'],3))"
  done
done

#!/bin/bash
# Short bench over precisions / kernels / poses (no CPU baseline), each step time-limited.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in ${CFGS:-bf16:proj fp16:proj bf16:grid fp16:grid fp32:grid}; do
  prec=${cfg%%:*}; mode=${cfg##*:}
  for extra in "" "--offset-pose"; do
    log=gpurun_out/bm_${prec}_${mode}${extra}.log
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --precision $prec --mode $mode $extra > $log 2>&1 || { cat $log; exit 7; }
    python -c "import json,sys; d=json.loads(open('$log').read().strip().splitlines()[-1]); r=d['roofline']; print('$prec $mode $extra', round(d['value']/1e6,2),'Mrays/s', round(d['ms_per_step'],3),'ms/step render', round(r['render_kernel_ms'],3),'proj', round(r['project_kernel_ms'],3),'frac', round(r['frac'],3))"
  done
done

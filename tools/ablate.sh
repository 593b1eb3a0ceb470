#!/bin/bash
# Diagnostic: bench the shipped library against variant builds (scenedino_amd/variants/*.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in $(seq ${REPS:-1}); do
for lib in scenedino_amd/libsdhip.so $(ls scenedino_amd/variants/*.so 2>/dev/null); do
  n=$(basename $lib .so)
  for prec in ${PRECS:-fp16}; do
    SDHIP_LIB=$lib timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline --precision $prec ${EXTRA} > gpurun_out/abl_${n}_$prec.log 2>&1 || { cat gpurun_out/abl_${n}_$prec.log; exit 7; }
    python -c "import json; d=json.loads(open('gpurun_out/abl_${n}_$prec.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$n', '$prec', 'render', round(r.get('render_kernel_ms', r['kernel_ms']),3),'ms', round(d['value']/1e6,2), 'Mrays/s')"
  done
done
done

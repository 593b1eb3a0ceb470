#!/bin/bash
# Diagnostic: C5 bench (field query / seg head kernel times) for the shipped library and
# every scenedino_amd/variants/*.so.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in scenedino_amd/libsdhip.so $(ls scenedino_amd/variants/*.so 2>/dev/null); do
  n=$(basename $lib .so)
  SDHIP_LIB=$lib timeout -k 10 200 python bench.py --config c5 --steps 10 --warmup 3 ${EXTRA} > gpurun_out/c5ab_$n.log 2>&1 || { tail -5 gpurun_out/c5ab_$n.log; exit 7; }
  python -c "import json; d=json.loads([l for l in open('gpurun_out/c5ab_$n.log') if l.startswith('{')][-1]); r=d['roofline']; print('$n', round(d['ms_per_step'],3), 'field', round(r['field_query_ms'],3), 'seg', round(r['kernel_ms'],3))"
done

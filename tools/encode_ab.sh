#!/bin/bash
# Diagnostic: interleaved `bench.py --config encode` runs of the shipped library and
# scenedino_amd/variants/$VARIANT.so (tools/build_variant.py), ms per pass per model.
set -o pipefail
mkdir -p gpurun_out/encab
for rep in 1 2 3; do
  for v in main ${VARIANT:-cvwt0}; do
    lib=""; [ $v != main ] && lib=scenedino_amd/variants/$v.so
    SDHIP_LIB=$lib timeout -k 10 300 python -u bench.py --config encode --no-cpu-baseline > gpurun_out/encab/$v.$rep.log 2>&1 || { tail -5 gpurun_out/encab/$v.$rep.log; exit 3; }
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/encab/$v.$rep.log') if l.startswith('{')][-1]); print('$v', {k: round(m['ms_per_pass'],4) for k,m in d['models'].items()})"
  done
done

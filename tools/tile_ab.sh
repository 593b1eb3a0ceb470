#!/bin/bash
# Diagnostic: render parity of every variant library (tests/test_gpu_parity.py through
# SDHIP_LIB) and the C2 bench A/B (tools/ablate.sh).  usage (on the GPU box):
#   REPS=2 tools/tile_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in $(ls scenedino_amd/variants/*.so 2>/dev/null); do
  n=$(basename $lib .so)
  SDHIP_LIB=$lib timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_parity.py -m gpu > gpurun_out/ab_parity_$n.log 2>&1 || { tail -30 gpurun_out/ab_parity_$n.log; exit 7; }
  tail -1 gpurun_out/ab_parity_$n.log
done
PRECS=${PRECS:-bf16} EXTRA="${EXTRA:---no-end-to-end}" bash tools/ablate.sh

#!/bin/bash
# Diagnostic: VALU / MFMA / LDS instruction counts of k_render_tile per ablation variant.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/abl_pmc
for lib in scenedino_amd/libsdhip.so $(ls scenedino_amd/variants/*.so 2>/dev/null); do
  n=$(basename $lib .so)
  SDHIP_LIB=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY -d gpurun_out/abl_pmc/$n -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-end-to-end ${EXTRA} > gpurun_out/abl_pmc/$n.log 2>&1 || { tail -5 gpurun_out/abl_pmc/$n.log; exit 3; }
  echo "== $n"; python3 tools/pmc_summary.py gpurun_out/abl_pmc/$n k_render_tile | tail -6
done

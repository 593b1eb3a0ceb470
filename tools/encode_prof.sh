#!/bin/bash
# Diagnostic: kernel trace of the ViT + DPT encode bench (rocprofv3 sqlite), one model per run;
# summarise with tools/trace_pass.py gpurun_out/encprof/<model>/run_results.db
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/encprof
export TMPDIR=/tmp
for m in ${MODELS:-vit-s16}; do
  timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/encprof/$m -o run -- \
    python bench.py --config encode --models $m --steps 10 --warmup 3 > gpurun_out/encprof/$m.log 2>&1 || exit 7
done

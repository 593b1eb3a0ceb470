#!/bin/bash
# Diagnostic: kernel trace + stats of the ViT encoder benches (rocprofv3), one model per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/vitprof
export TMPDIR=/tmp
for m in ${MODELS:-vit-s16 dinov2-b14}; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/vitprof/$m -o run -- \
    python bench.py --config vit --models $m --steps 10 --warmup 3 > gpurun_out/vitprof/$m.log 2>&1 || exit 7
done

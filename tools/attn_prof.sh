#!/bin/bash
# rocprofv3 kernel stats of the ViT-B/8 pass with each attention kernel forced
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/attnprof
mkdir -p $O
for m in lds dir; do
  SD_ATTN=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$m -o run --output-format csv -- python3 bench.py --config vit --models ${MODELS:-vit-b8} --steps 10 --warmup 2 > $O/$m.log 2>&1 || { tail -20 $O/$m.log; exit 3; }
  f=$(find $O/$m -name "*kernel_stats.csv" | head -1)
  echo "== $m"; head -8 "$f" | cut -d, -f1-8
done

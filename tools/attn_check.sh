#!/bin/bash
# attention A/B: ViT tests, then the ViT bench with each attention kernel forced
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/attn
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_vit.py tests/test_encoder.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 2; }
tail -2 $O/pytest.log
for m in auto lds dir; do
  SD_ATTN=$([ $m = auto ] && echo "" || echo $m) timeout -k 10 300 python bench.py --config vit > $O/vit_$m.log 2>&1 || { tail -20 $O/vit_$m.log; exit 3; }
  echo "== $m"; grep "^{" $O/vit_$m.log | cut -c1-1500
done

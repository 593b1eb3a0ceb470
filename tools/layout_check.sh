#!/bin/bash
# full GPU suite, then C2 and train benches with both grid layouts
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/layout
mkdir -p $O
bash tools/gpu_tests.sh || exit 2
for L in nhwc nchw; do
  timeout -k 10 300 python bench.py --no-end-to-end --no-cpu-baseline --grid-layout $L > $O/c2_$L.log 2>&1 || { tail -20 $O/c2_$L.log; exit 3; }
  timeout -k 10 300 python bench.py --config train --steps 10 --warmup 3 --grid-layout $L > $O/train_$L.log 2>&1 || { tail -20 $O/train_$L.log; exit 4; }
  echo "== $L"; grep '^{' $O/c2_$L.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2', round(d['ms_per_step'],4), {k: round(v['render_kernel_ms'],4) for k,v in d['poses'].items()}, {k: round(v['project_kernel_ms'],4) for k,v in d['poses'].items()})"
  grep '^{' $O/train_$L.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('train', round(d['ms_per_step'],4))"
done

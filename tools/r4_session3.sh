#!/bin/bash
# Round-4 GPU session 3: the GPU suite on the ring-default library, the default-graph train
# step, ViT-S/16 SQ counter passes, the C2 traffic passes (k_project_lds + k_render_tile).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/r4s3
mkdir -p $O
t() { timeout -k 10 "$@"; }
t 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 3; }
tail -3 $O/pytest_gpu.log
t 300 python -u bench.py --config train --steps 20 --warmup 3 > $O/train.log 2>&1 || { tail -30 $O/train.log; exit 4; }
grep '^{' $O/train.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('train', d['ms_per_step'], d['step_issue'])"
t 400 tools/r4_vit_pmc.sh > $O/vitpmc.log 2>&1 || { tail -30 $O/vitpmc.log; exit 5; }
cat gpurun_out/r4vitpmc/summary.txt | head -60
t 600 tools/r4_pmc_c2.sh > $O/c2pmc.log 2>&1 || { tail -30 $O/c2pmc.log; exit 6; }
cat gpurun_out/r4pmc/r4_traffic_offset.json
echo r4s3-done

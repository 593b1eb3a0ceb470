#!/bin/bash
# Round-4 GPU session 22: C5 voxel query in chunks, the seg head of chunk i on a side stream
# beside the field query of chunk i + 1 -- parity, then bench c5 at 1 / 2 / 4 / 8 chunks.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/r4s22
mkdir -p $O
t() { timeout -k 10 "$@"; }
t 400 python -u -m pytest tests/test_seg.py -m gpu -q --timeout 200 --timeout-method thread -k "voxel_query" > $O/pytest.log 2>&1 || { grep -E "FAIL|Error|assert" $O/pytest.log | tail -30; exit 3; }
tail -1 $O/pytest.log
for rep in 1 2; do
  for k in 1 2 4 8; do
    SCENEDINO_AMD_VOXEL_CHUNKS=$k t 300 python -u bench.py --config c5 --no-cpu-baseline > $O/c5_k$k.$rep.log 2>&1 || { tail -20 $O/c5_k$k.$rep.log; exit 5; }
    python3 -c "import json; d=json.loads([l for l in open('$O/c5_k$k.$rep.log') if l.startswith('{')][-1]); print('chunks $k', round(d['ms_per_step'],4))"
  done
done
echo r4s22-done

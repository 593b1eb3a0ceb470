#!/bin/bash
# Seg head iteration: GPU tests, kernel time (shipped + variants), phase profile.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/segi
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_seg.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 2; }
tail -1 $O/pytest.log
timeout -k 10 120 python tools/seg_time.py 2>&1 | grep k_seg || exit 3
for v in $VARIANTS; do SDHIP_LIB=scenedino_amd/_exp/$v.so timeout -k 10 120 python tools/seg_time.py 2>&1 | grep k_seg || exit 4; done
SDHIP_LIB=scenedino_amd/_exp/prof.so timeout -k 10 120 python tools/seg_prof.py 2>&1 | grep -v amdgpu.ids || exit 5

#!/bin/bash
# Round-4 GPU session 7: conv ring depth (6 vs 4 stages) and 256-deep split-K tiles (on / off)
# A/B on the ViT and encode passes, parity of the shipped build, per-kernel encode trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/r4s7
mkdir -p $O
t() { timeout -k 10 "$@"; }
t 300 python -u -m pytest tests/test_vit.py tests/test_dpt.py tests/test_encoder.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 3; }
grep -E "passed|failed" $O/pytest.log | tail -2
for rep in 1 2; do
for v in main cv4 nosk256; do
  lib=""; [ $v != main ] && lib=scenedino_amd/variants/$v.so
  for c in vit encode; do
    SDHIP_LIB=$lib t 300 python -u bench.py --config $c > $O/${c}_$v.log 2>&1 || { tail -20 $O/${c}_$v.log; exit 5; }
    python3 -c "import json,sys; d=json.loads([l for l in open('$O/${c}_$v.log') if l.startswith('{')][-1]); print('$c $v', {m: round(v['ms_per_pass'],4) for m,v in d['models'].items()})"
  done
done
done
t 240 rocprofv3 --kernel-trace -d $O/enc -o run -- python3 bench.py --config encode --models vit-s16 --steps 10 --warmup 3 > $O/enc.log 2>&1 || { tail -20 $O/enc.log; exit 6; }
db=$(find $O/enc -name "*.db" | head -1)
python3 tools/trace_pass.py $db k_patchify --list > $O/enc_trace.txt 2>&1; head -24 $O/enc_trace.txt
echo r4s7-done

#!/bin/bash
# Round-4 GPU session 6: the DPT's 256-row LDS-DMA tiles (sdhip_conv.hip, 128-row tiles + residual units): parity, encode A/B
# against the k_gemm path (SD_CONV_BIG=0), per-kernel trace of one encode pass.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/r4s6
mkdir -p $O
t() { timeout -k 10 "$@"; }
t 300 python -u -m pytest tests/test_dpt.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_dpt.log 2>&1 || { tail -40 $O/pytest_dpt.log; exit 3; }
grep -E "passed|failed" $O/pytest_dpt.log | tail -2
for rep in 1 2; do
for v in big old; do
  e=1; [ $v = old ] && e=0
  SD_CONV_BIG=$e t 300 python -u bench.py --config encode > $O/encode_$v.log 2>&1 || { tail -20 $O/encode_$v.log; exit 5; }
  python3 -c "import json,sys; d=json.loads([l for l in open('$O/encode_$v.log') if l.startswith('{')][-1]); print('$v', {m: round(v['ms_per_pass'],4) for m,v in d['models'].items()})"
done
done
t 240 rocprofv3 --kernel-trace -d $O/enc -o run -- python3 bench.py --config encode --models vit-s16 --steps 10 --warmup 3 > $O/enc.log 2>&1 || { tail -20 $O/enc.log; exit 6; }
db=$(find $O/enc -name "*.db" | head -1)
python3 tools/trace_pass.py $db k_patchify --list > $O/enc_trace.txt 2>&1; head -16 $O/enc_trace.txt; tail -12 $O/enc_trace.txt
echo r4s6-done

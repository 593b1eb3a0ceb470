#!/bin/bash
# Round-4 GPU session 17: the DPT level fronts on side streams beside the ViT (encoder
# parity incl. one-stream bit equality, eager and graphed), encode / end-to-end timings
# with overlap on and off (DINOv2Module.overlap_levels), interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export PYTHONDONTWRITEBYTECODE=1 TMPDIR=/tmp
O=gpurun_out/r4s17
mkdir -p $O
t() { timeout -k 10 "$@"; }
t 400 python -u -m pytest tests/test_encoder.py tests/test_dpt.py tests/test_vit.py -m gpu -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" $O/pytest.log | tail -30; exit 3; }
grep -E "passed|failed" $O/pytest.log | tail -2
for rep in 1 2; do
  for ov in 1 0; do
    SCENEDINO_AMD_DPT_OVERLAP=$ov t 300 python -u bench.py --config encode > $O/encode_$ov$rep.log 2>&1 || { tail -20 $O/encode_$ov$rep.log; exit 5; }
    python3 -c "import json,sys; d=json.loads([l for l in open('$O/encode_$ov$rep.log') if l.startswith('{')][-1]); print('encode overlap=$ov', {m: round(v['ms_per_pass'],4) for m,v in d['models'].items()})"
  done
done
t 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/c2.log 2>&1 || { tail -20 $O/c2.log; exit 6; }
python3 -c "import json; d=json.loads([l for l in open('$O/c2.log') if l.startswith('{')][-1]); print('c2', round(d['ms_per_step'],4), 'e2e', d.get('end_to_end',{}).get('ms_per_frame'))"
echo r4s17-done

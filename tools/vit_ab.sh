set -o pipefail
mkdir -p gpurun_out/vab
V=scenedino_amd/variants
SDHIP_LIB=$PWD/$V/libsdhip_lnq.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_vit.py -m gpu > gpurun_out/vab/parity.log 2>&1 || { tail -30 gpurun_out/vab/parity.log; exit 3; }
tail -1 gpurun_out/vab/parity.log
for rep in 1 2 3; do for n in lnqbase lnq; do
SDHIP_LIB=$PWD/$V/libsdhip_$n.so timeout -k 10 200 python bench.py --config vit --models vit-s16,dinov2-b14 > gpurun_out/vab/$n.$rep.log 2>&1 || { tail -20 gpurun_out/vab/$n.$rep.log; exit 4; }
python -c "import json; d=json.loads([l for l in open('gpurun_out/vab/$n.$rep.log') if l.startswith('{')][0]); print('$n', {k: round(v['ms_per_pass'],4) for k,v in d['models'].items()})"
done; done

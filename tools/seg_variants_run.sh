set -o pipefail
export PYTHONDONTWRITEBYTECODE=1
mkdir -p gpurun_out/segx
timeout -k 10 120 python tools/seg_time.py > gpurun_out/segx/t.log 2>&1 || { cat gpurun_out/segx/t.log; exit 2; }
for v in ${VARIANTS:-exp1 w4 nt1 nt1w4}; do SDHIP_LIB=scenedino_amd/_exp/$v.so timeout -k 10 120 python tools/seg_time.py >> gpurun_out/segx/t.log 2>&1 || { cat gpurun_out/segx/t.log; exit 3; }; done
cat gpurun_out/segx/t.log

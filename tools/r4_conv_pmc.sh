#!/bin/bash
# Round-4 DPT convolution diagnosis: SQ / TCC / GRBM counter passes (separate runs, kernel
# trace only) of the ViT-S/16 + DPT encode pass, summarised per kernel (tools/pmc_summary.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/r4convpmc
mkdir -p $O
B="bench.py --config encode --models vit-s16 --steps 3 --warmup 1"
P1="GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
P2="SQ_WAVES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD"
P3="TCC_HIT_sum TCC_MISS_sum"
P4="FETCH_SIZE"
i=0
for p in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $p -d $O/pmc$i -o run --output-format csv -- python3 $B > $O/pmc$i.log 2>&1 || { tail -20 $O/pmc$i.log; exit 2; }
done
python3 tools/pmc_summary.py $O k_conv_big k_gemm k_lngemm k_attn > $O/summary.txt 2>&1; cat $O/summary.txt
echo convpmc-done

#!/bin/bash
# Round-4 GPU session 23: k_render_tile stall / LDS counters (offset pose) on the shipped
# library, the three SQ passes of tools/pmc_tile.sh (separate runs), for the round-3 vs
# round-4 comparison in DESIGN §5.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/r4s23
mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_LDS"
P3="SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_INSTS_SMEM SQ_THREAD_CYCLES_VALU SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_WAVES"
i=0
for pmc in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $pmc -d $O/main/pmc$i -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-end-to-end --offset-pose > $O/pmc$i.log 2>&1 || { tail -5 $O/pmc$i.log; exit 3; }
done
python3 tools/pmc_summary.py $O/main k_render_tile > $O/summary.txt && cat $O/summary.txt
echo r4s23-done

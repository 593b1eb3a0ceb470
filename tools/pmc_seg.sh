#!/bin/bash
# Diagnostic: stall breakdown of k_seg_head (tools/seg_time.py, the C5 launch) in three PMC
# passes, for the shipped library and the given scenedino_amd/_exp/*.so variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONDONTWRITEBYTECODE=1
O=gpurun_out/pmc_seg
mkdir -p $O
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_LDS"
P3="SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT"
for lib in scenedino_amd/libsdhip.so "$@"; do
  n=$(basename $lib .so)
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $O/$n/trace -o run --output-format csv -- python3 tools/seg_time.py > $O/$n.trace.log 2>&1 || { tail -5 $O/$n.trace.log; exit 2; }
  i=0
  for pmc in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    SDHIP_LIB=$lib timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $pmc -d $O/$n/pmc$i -o run --output-format csv -- python3 tools/seg_time.py > $O/$n.pmc$i.log 2>&1 || { tail -5 $O/$n.pmc$i.log; exit 3; }
  done
  echo "== $n"; python3 tools/pmc_summary.py $O/$n k_seg_head
done

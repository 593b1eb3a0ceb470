#!/bin/bash
# Build timing-experiment variants of libsdhip.so that differ only in sdhip_seg.hip's macros
# (usage: tools/seg_variants.sh NAME "-DMACRO=..." ...); outputs scenedino_amd/_exp/NAME.so
set -e
cd "$(dirname "$0")/.."
python -m scenedino_amd.build > /dev/null
F="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -DSD_FASTPE=0 -Wno-unused-result -mllvm -amdgpu-mfma-vgpr-form=1 -fno-slp-vectorize"
while [ $# -gt 0 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc $F $flags -c scenedino_amd/csrc/sdhip_seg.hip -o /tmp/seg_$name.o
  objs=$(ls scenedino_amd/_obj/*.o | grep -v sdhip_seg)
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o scenedino_amd/_exp/$name.so $objs /tmp/seg_$name.o
done

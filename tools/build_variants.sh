#!/bin/bash
# Diagnostic: build variant libraries (same sources, different -D switches) into
# scenedino_amd/variants/<name>.so for tools/ablate.sh.  usage: build_variants.sh name:"-DA=1 -DB=2" ...
set -e
cd "$(dirname "$0")/.."
mkdir -p scenedino_amd/variants
for spec in "$@"; do
  name=${spec%%:*}; defs=${spec#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared \
    -DSD_FASTPE=0 -Wno-unused-result -mllvm -amdgpu-mfma-vgpr-form=1 -fno-slp-vectorize $defs \
    -o scenedino_amd/variants/$name.so scenedino_amd/csrc/sdhip_rays.hip \
    scenedino_amd/csrc/sdhip_field.hip scenedino_amd/csrc/sdhip_proj.hip &
done
wait
ls -la scenedino_amd/variants

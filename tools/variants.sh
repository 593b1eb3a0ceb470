#!/bin/bash
# Build alternative sdhip_field.hip sources into scenedino_amd/variants/libsdhip_<name>.so
# (diagnostic A/B builds, loaded via SDHIP_LIB).  usage: tools/variants.sh name=path.hip ...
cd "$(dirname "$0")/.."
mkdir -p scenedino_amd/variants
for spec in "$@"; do
  name=${spec%%=*}; src=${spec#*=}
  cp "$src" scenedino_amd/csrc/_variant_$name.hip
  ( /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared \
    -DSD_FASTPE=0 -Wno-unused-result -o scenedino_amd/variants/libsdhip_$name.so \
    scenedino_amd/csrc/sdhip_rays.hip scenedino_amd/csrc/_variant_$name.hip;
    rm -f scenedino_amd/csrc/_variant_$name.hip ) &
done
wait
ls -la scenedino_amd/variants

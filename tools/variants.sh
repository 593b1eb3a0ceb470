#!/bin/bash
# Build diagnostic A/B variants of libsdhip.so with extra compiler flags into
# scenedino_amd/variants/libsdhip_<name>.so (loaded via SDHIP_LIB by tools/ablate.sh).
# usage: tools/variants.sh 'name=-DFOO=1 -DBAR=2' ...
cd "$(dirname "$0")/.."
mkdir -p scenedino_amd/variants
FLAGS=$(python -c "import sys; sys.path.insert(0,'scenedino_amd'); import build; print(' '.join(build.FLAGS))")
SRCS=$(python -c "import sys; sys.path.insert(0,'scenedino_amd'); import build; print(' '.join('scenedino_amd/'+s for s in build.SOURCES))")
for spec in "$@"; do
  name=${spec%%=*}; extra=${spec#*=}
  /opt/rocm/bin/hipcc $FLAGS -shared $extra -o scenedino_amd/variants/libsdhip_$name.so $SRCS &
done
wait
ls -la scenedino_amd/variants

#!/bin/bash
# Build engine variants that differ only by -D flags, for timing comparisons on the GPU box.
# usage: tools/build_variants.sh NAME:"-DFLAG=V -DFLAG2" ...   -> build/var/libmfg_hip_NAME.so
set -e
cd "$(dirname "$0")/.."
mkdir -p build/var
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -shared -fPIC $flags \
    -o build/var/libmfg_hip_$name.so marl-factory-grid_amd/csrc/mfg_engine.hip &
done
wait
ls build/var

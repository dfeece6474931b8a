#!/bin/bash
# Timing-only ablation builds of the engine (results are WRONG by construction; never used for parity).
# usage: tools/build_ablation.sh [VARIANT ...]   (default: NOSWAP NODEBT NOOBS)
set -e
cd "$(dirname "$0")/.."
mkdir -p build/ablate
VARS=${*:-NOSWAP NODEBT NOOBS}
for v in $VARS; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -shared -fPIC -DMFG_ABLATE_$v \
    -o build/ablate/libmfg_hip_$v.so marl-factory-grid_amd/csrc/mfg_engine.hip &
done
wait
ls build/ablate

#!/bin/bash
# Timing-only ablation builds of the engine (results are WRONG by construction; never used for parity).
set -e
cd "$(dirname "$0")/.."
mkdir -p build/ablate
for v in NOSWAP NODEBT NOOBS; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -shared -fPIC -DMFG_ABLATE_$v \
    -o build/ablate/libmfg_hip_$v.so marl-factory-grid_amd/csrc/mfg_engine.hip &
done
wait
ls -la build/ablate

#!/bin/bash
# Exact k_replay swap-block variants for A/B timing: build/ablate/libmfg_hip_RPV<n>.so with -DMFG_RPV=<n>.
set -e
cd "$(dirname "$0")/.."
mkdir -p build/ablate
for v in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -shared -fPIC -DMFG_RPV=$v \
    -o build/ablate/libmfg_hip_RPV$v.so marl-factory-grid_amd/csrc/mfg_engine.hip &
done
wait

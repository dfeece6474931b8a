#!/bin/bash
# Exact engine variants for A/B timing (tools/ab_run.sh): build/ablate/libmfg_hip_VARIANT.so with -DMFG_VARIANT.
set -e
cd "$(dirname "$0")/.."
mkdir -p build/ablate
for v in "$@"; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -shared -fPIC -DMFG_$v \
    -o build/ablate/libmfg_hip_$v.so marl-factory-grid_amd/csrc/mfg_engine.hip &
done
wait

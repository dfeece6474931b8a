#!/bin/bash
# Timing-only ablation builds of the engine (results are WRONG by construction; never used for parity).
# usage: tools/build_ablation.sh [VARIANT ...]   (default: NOSWAP NODEBT NOOBS)
set -e
cd "$(dirname "$0")/.."
mkdir -p build/ablate
for v in ${*:-NOSWAP NODEBT NOOBS}; do
  ./tools/build_lib.sh build/ablate/libmfg_hip_$v.so -DMFG_ABLATE_$v
done
ls build/ablate

#!/bin/bash
# Build the engine library: the host unit and the four observation-render units compile in parallel, then link.
# usage: tools/build_lib.sh OUT.so [extra hipcc flags, e.g. -DMFG_RPV=3]
set -e
cd "$(dirname "$0")/.."
OUT=$1; shift
OBJ=$(mktemp -d /tmp/mfg_build.XXXXXX)
CSRC=marl-factory-grid_amd/csrc
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC $*"
pids=()
for u in mfg_engine mfg_obs_a mfg_obs_b mfg_obs_c mfg_obs_d mfg_obs_e mfg_obs_f mfg_learn; do
  /opt/rocm/bin/hipcc $FLAGS -c -o $OBJ/$u.o $CSRC/$u.hip & pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT" $OBJ/*.o
rm -rf $OBJ

#!/bin/bash
# Render variants for A/B timing of the C2/C3 render (ray lengths 4-8 live in mfg_obs_a.hip): only that unit is
# recompiled with the variant's flags and linked with the in-tree build's other objects (build/obj, refreshed by
# __graft_entry__.build_hip()).
# usage: tools/build_obs_variant.sh NAME=FLAGS ...   -> build/ablate/libmfg_hip_NAME.so
set -e
cd "$(dirname "$0")/.."
CSRC=marl-factory-grid_amd/csrc
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC"
mkdir -p build/ablate
pids=()
for arg in "$@"; do
  name=${arg%%=*}; flags=${arg#*=}
  /opt/rocm/bin/hipcc $FLAGS $flags -c -o build/obj/obs_a_$name.o $CSRC/mfg_obs_a.hip & pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
for arg in "$@"; do
  name=${arg%%=*}
  objs=""
  for u in mfg_engine mfg_obs_b mfg_obs_c mfg_obs_d mfg_obs_e mfg_obs_f mfg_learn; do objs="$objs build/obj/$u.o"; done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/ablate/libmfg_hip_$name.so build/obj/obs_a_$name.o $objs
done
ls -la build/ablate

#!/bin/bash
# Render variants for A/B timing: only the render units in $OBS_UNITS (default mfg_obs_a: ray lengths 4-8, C2/C3; C4's
# 10-point rays are in mfg_obs_b, C5's 18 in mfg_obs_c) are recompiled with the variant's flags and linked with the
# in-tree build's other objects (build/obj, refreshed by __graft_entry__.build_hip()).
# usage: [OBS_UNITS="mfg_obs_a mfg_obs_b"] tools/build_obs_variant.sh NAME=FLAGS ...   -> build/ablate/libmfg_hip_NAME.so
set -e
cd "$(dirname "$0")/.."
CSRC=marl-factory-grid_amd/csrc
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC"
VU=${OBS_UNITS:-mfg_obs_a}
mkdir -p build/ablate
pids=()
for arg in "$@"; do
  name=${arg%%=*}; flags=${arg#*=}
  for u in $VU; do
    /opt/rocm/bin/hipcc $FLAGS $flags -c -o build/obj/${u}_$name.o $CSRC/$u.hip & pids+=($!)
  done
done
for p in "${pids[@]}"; do wait $p; done
for arg in "$@"; do
  name=${arg%%=*}
  objs=""
  for u in mfg_engine mfg_obs_a mfg_obs_b mfg_obs_c mfg_obs_d mfg_obs_e mfg_obs_f mfg_learn; do
    if [[ " $VU " == *" $u "* ]]; then objs="$objs build/obj/${u}_$name.o"; else objs="$objs build/obj/$u.o"; fi
  done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/ablate/libmfg_hip_$name.so $objs
done
ls -la build/ablate

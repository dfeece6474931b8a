#!/bin/bash
# Engine variants that change only the host unit (mfg_engine.hip: k_logic, k_replay*, resets): the four render
# units are compiled once with the default flags (build/obj) and linked to each variant's host unit.
# usage: tools/build_engine_variant.sh NAME=FLAGS ...   -> build/ablate/libmfg_hip_NAME.so
set -e
cd "$(dirname "$0")/.."
CSRC=marl-factory-grid_amd/csrc
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC"
mkdir -p build/obj build/ablate
for u in mfg_obs_a mfg_obs_b mfg_obs_c mfg_obs_d mfg_obs_e mfg_obs_f mfg_learn; do
  if [ ! -f build/obj/$u.o ] || [ $CSRC/mfg_kernels.h -nt build/obj/$u.o ] || [ $CSRC/$u.hip -nt build/obj/$u.o ]; then
    /opt/rocm/bin/hipcc $FLAGS -c -o build/obj/$u.o $CSRC/$u.hip &
  fi
done
pids=()
for arg in "$@"; do
  name=${arg%%=*}; flags=${arg#*=}
  /opt/rocm/bin/hipcc $FLAGS $flags -c -o build/obj/engine_$name.o $CSRC/mfg_engine.hip & pids+=($!)
done
wait
for arg in "$@"; do
  name=${arg%%=*}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o build/ablate/libmfg_hip_$name.so build/obj/engine_$name.o \
    build/obj/mfg_obs_a.o build/obj/mfg_obs_b.o build/obj/mfg_obs_c.o build/obj/mfg_obs_d.o build/obj/mfg_obs_e.o build/obj/mfg_obs_f.o build/obj/mfg_learn.o
done
ls -la build/ablate

#!/bin/bash
# Engine variants for A/B timing (tools/ab_run.sh): build/ablate/libmfg_hip_NAME.so from "NAME=FLAGS" arguments,
# e.g. tools/build_variant.sh RPV7=-DMFG_RPV=7 OVL0=-DMFG_RESET_OVERLAP=0 (one variant at a time: each build is
# already 5 parallel compiles).
set -e
cd "$(dirname "$0")/.."
mkdir -p build/ablate
for arg in "$@"; do
  name=${arg%%=*}; flags=${arg#*=}
  ./tools/build_lib.sh build/ablate/libmfg_hip_$name.so $flags
done

#!/bin/bash
# Run on the GPU box: time the baseline and each ablation variant (timing only).
# usage: tools/ablate_run.sh [VARIANT ...]
cd "$(dirname "$0")/.."
VARS=${*:-NOSWAP NODEBT NOOBS}
for v in BASE $VARS; do
  if [ $v = BASE ]; then unset MFG_HIP_LIB; else export MFG_HIP_LIB=$PWD/build/ablate/libmfg_hip_$v.so; fi
  echo "== $v"
  timeout -k 10 300 python bench.py --steps 48 --warmup 8 --no-cpu-baseline | python -c "import json,sys; d=json.loads(sys.stdin.readlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['mean_launch_ms'])" || exit 1
done

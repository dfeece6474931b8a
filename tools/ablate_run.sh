#!/bin/bash
# Run on the GPU box: time the baseline and each ablation variant (timing only; ablated builds compute
# wrong results by construction). Prints env-steps/s, ms/step and the per-kernel mean launch times.
# usage: tools/ablate_run.sh [VARIANT ...]
cd "$(dirname "$0")/.."
VARS=${*:-NOSWAP NODEBT NOOBS}
for v in BASE $VARS; do
  if [ $v = BASE ]; then unset MFG_HIP_LIB; else export MFG_HIP_LIB=$PWD/build/ablate/libmfg_hip_$v.so; fi
  timeout -k 10 300 python bench.py --steps 400 --warmup 100 --no-cpu-baseline --alt-steps 0 --packed-steps 0 | python -c "
import json,sys; d=json.loads(sys.stdin.readlines()[-1]); k=d['roofline'].get('kernels',{})
print('$v', d['value'], d['ms_per_step'], {n: v['mean_launch_ms'] for n, v in k.items()})" || exit 1
done

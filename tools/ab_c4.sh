#!/bin/bash
# A/B on C4 (alltest16, 32,768 envs): tools/ab_c4.sh VARIANT (build/ablate/libmfg_hip_VARIANT.so) vs in-tree.
cd "$GRAFT_REPO_ROOT" || exit 1
for v in base "$@"; do
  lib=""; [ "$v" != base ] && lib="build/ablate/libmfg_hip_$v.so"
  MFG_HIP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --config alltest16.yaml --batch 32768 \
    --steps 200 --warmup 50 --alt-steps 0 --packed-steps 0 > gpurun_out/abc4_$v.json 2>/dev/null || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/abc4_$v.json'))
print('c4 $v', round(d['value']/1e6,3), {k: v['mean_launch_ms'] for k, v in d['roofline']['kernels'].items()})"
done

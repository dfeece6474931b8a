#!/bin/bash
# Parity subset (fixture replay) for engine variants, then their A/B timing: tools/gpu_bisect.sh VARIANT...
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in "$@"; do
  MFG_HIP_LIB=build/ablate/libmfg_hip_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py \
    tests/test_gpu_timed_path.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/bis_$v.log 2>&1
  echo "$v: $(tail -1 gpurun_out/bis_$v.log)"
done
for r in 1 2; do
  for v in base "$@"; do
    lib=""; [ "$v" != base ] && lib="build/ablate/libmfg_hip_$v.so"
    MFG_HIP_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --alt-steps 0 \
      --packed-steps 0 --steps 800 --warmup 200 > gpurun_out/ab_$v.json 2>/dev/null || exit 1
    python -c "
import json; d=json.load(open('gpurun_out/ab_$v.json'))
print('$v', round(d['value']/1e6,2), {k: v['mean_launch_ms'] for k, v in d['roofline']['kernels'].items()})"
  done
done

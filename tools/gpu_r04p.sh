#!/bin/bash
# Render store policy A/B: in-tree (non-temporal obs stores) vs PMW (plain stores in the multi-wave render, f32 and
# f64) vs NT0 (plain f64 stores in every render): C3 f64/f32, C4 f64/f32, C5 f64 (short).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
run() {  # tag lib args...
  local tag=$1 lib=$2; shift 2
  MFG_HIP_LIB=$lib timeout -k 10 400 python bench.py --no-cpu-baseline --alt-steps 0 --packed-steps 0 "$@" \
    > gpurun_out/r04p_$tag.json 2> gpurun_out/r04p_$tag.err || { tail -5 gpurun_out/r04p_$tag.err; return 1; }
  python - $tag <<'PY'
import json, sys
t = sys.argv[1]
d = json.load(open(f'gpurun_out/r04p_{t}.json'))
k = d['roofline']['kernels']
print(t, round(d['value']), round(d['ms_per_step'], 4), {n: round(x['mean_launch_ms'], 4) for n, x in k.items() if 'mean_launch_ms' in x and x['mean_launch_ms'] > 0.02})
PY
}
for v in base PMW NT0; do
  lib=""; [ $v != base ] && lib=build/ablate/libmfg_hip_$v.so
  run c4f64_$v "$lib" --config alltest16.yaml --batch 32768 --steps 200 --warmup 50 || exit 1
  run c4f32_$v "$lib" --config alltest16.yaml --batch 32768 --steps 200 --warmup 50 --obs-dtype f32 || exit 1
  run c3f64_$v "$lib" --steps 400 --warmup 100 || exit 1
  run c5f64_$v "$lib" --config grid128_64.yaml --batch 131072 --fuse 1 --steps 4 --warmup 2 || exit 1
done

#!/bin/bash
# SPLIT store variant (plain stores only on a row's partial end lines) vs in-tree, 2 rounds: C3 f64/f32, C5 f64.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
run() {  # tag lib args...
  local tag=$1 lib=$2; shift 2
  MFG_HIP_LIB=$lib timeout -k 10 400 python bench.py --no-cpu-baseline --alt-steps 0 --packed-steps 0 "$@" \
    > gpurun_out/r04r_$tag.json 2> gpurun_out/r04r_$tag.err || { tail -5 gpurun_out/r04r_$tag.err; return 1; }
  python - $tag <<'PY'
import json, sys
t = sys.argv[1]
d = json.load(open(f'gpurun_out/r04r_{t}.json'))
k = d['roofline']['kernels']
print(t, round(d['value']), round(d['ms_per_step'], 4), {n: round(x['mean_launch_ms'], 4) for n, x in k.items() if 'mean_launch_ms' in x and x['mean_launch_ms'] > 0.02})
PY
}
for r in 1 2; do
for v in base ${VARIANTS:-SPLIT}; do
  lib=""; [ $v != base ] && lib=build/ablate/libmfg_hip_$v.so
  run c3f64_${v}_$r "$lib" --steps 400 --warmup 100 || exit 1
  run c3f32_${v}_$r "$lib" --steps 400 --warmup 100 --obs-dtype f32 || exit 1
  [ $r = 1 ] && { run c5f64_${v} "$lib" --config grid128_64.yaml --batch 131072 --fuse 1 --steps 4 --warmup 2 || exit 1; }
done
done

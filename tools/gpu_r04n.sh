#!/bin/bash
# C4 A/B: per-step replay (in-tree) vs one replay per call (RE0), 2 alternating rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for r in 1 2; do
  for v in base RE0; do
    lib=""; [ $v != base ] && lib=build/ablate/libmfg_hip_$v.so
    MFG_HIP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --config alltest16.yaml --batch 32768 --steps 200 --warmup 50 \
      --alt-steps 0 --packed-steps 0 > gpurun_out/r04n_c4_${v}_$r.json 2> gpurun_out/r04n_c4_${v}_$r.err || { tail -5 gpurun_out/r04n_c4_${v}_$r.err; exit 1; }
    python - $v $r <<'PY'
import json, sys
v, r = sys.argv[1:3]
d = json.load(open(f'gpurun_out/r04n_c4_{v}_{r}.json'))
k = d['roofline']['kernels']
print('c4', v, r, round(d['value']), round(d['ms_per_step'], 4), {n: round(x['mean_launch_ms'], 4) for n, x in k.items() if 'mean_launch_ms' in x})
PY
  done
done

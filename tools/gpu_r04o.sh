#!/bin/bash
# Render store ablation (timing only: values computed, not stored) at C3 (f64) and C4 (f64): is k_obs store-bound?
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in base ${VARIANTS:-NOST}; do
  lib=""; [ $v != base ] && lib=build/ablate/libmfg_hip_$v.so
  MFG_HIP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --steps 400 --warmup 100 --alt-steps 0 --packed-steps 0 \
    > gpurun_out/r04o_c3_$v.json 2> gpurun_out/r04o_c3_$v.err || { tail -5 gpurun_out/r04o_c3_$v.err; exit 1; }
  MFG_HIP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --config alltest16.yaml --batch 32768 --steps 200 --warmup 50 \
    --alt-steps 0 --packed-steps 0 > gpurun_out/r04o_c4_$v.json 2> gpurun_out/r04o_c4_$v.err || { tail -5 gpurun_out/r04o_c4_$v.err; exit 1; }
  python - $v <<'PY'
import json, sys
v = sys.argv[1]
for c in ('c3', 'c4'):
    d = json.load(open(f'gpurun_out/r04o_{c}_{v}.json'))
    k = d['roofline']['kernels']
    print(c, v, round(d['value']), round(d['ms_per_step'], 4), {n: round(x['mean_launch_ms'], 4) for n, x in k.items() if 'mean_launch_ms' in x})
PY
done

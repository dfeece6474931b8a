#!/bin/bash
# k_logic<FULL> stages the MT/perm tail only where a RespawnDirt spawn fires: parity subset, then C2/C4 A/B
# against the previous library (build/ablate/libmfg_hip_OLD.so).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests \
  > gpurun_out/r04i_tests.txt 2>&1 \
  || { tail -30 gpurun_out/r04i_tests.txt; exit 1; }
tail -3 gpurun_out/r04i_tests.txt
for r in 1 2; do
  for v in OLD new; do
    lib=""; [ $v = OLD ] && lib=build/ablate/libmfg_hip_OLD.so
    MFG_HIP_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --config rooms4.yaml --batch 4096 --steps 400 --warmup 100 \
      --alt-steps 0 --packed-steps 0 > gpurun_out/r04i_c2_${v}_$r.json 2> gpurun_out/r04i_c2_${v}_$r.err || { tail -5 gpurun_out/r04i_c2_${v}_$r.err; exit 1; }
    MFG_HIP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --config alltest16.yaml --batch 32768 --steps 200 --warmup 50 \
      --alt-steps 0 --packed-steps 0 > gpurun_out/r04i_c4_${v}_$r.json 2> gpurun_out/r04i_c4_${v}_$r.err || { tail -5 gpurun_out/r04i_c4_${v}_$r.err; exit 1; }
    python - $v $r <<'PY'
import json, sys
v, r = sys.argv[1:3]
for c in ('c2', 'c4'):
    d = json.load(open(f'gpurun_out/r04i_{c}_{v}_{r}.json'))
    k = d['roofline']['kernels']
    print(c, v, r, round(d['value']), round(d['ms_per_step'], 4), {n: round(x['mean_launch_ms'], 4) for n, x in k.items() if 'mean_launch_ms' in x})
PY
  done
done

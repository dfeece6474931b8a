#!/bin/bash
# GPU suite (step-prefix record layout, chunked reset draws, replay2 consumer prefetch), C4 reset-draws A/B,
# C5 replay2 A/B, A2C loop GRU window modes, C3 bench.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/t_r03i.log 2>&1 || { tail -30 gpurun_out/t_r03i.log; exit 1; }
tail -1 gpurun_out/t_r03i.log
show() { python -c "
import json,sys; d=json.load(open(sys.argv[1]))
print(sys.argv[2], round(d['value']/1e6,4), d['ms_per_step'], {k: (v['launches'], v['mean_launch_ms']) for k, v in d['roofline']['kernels'].items() if v['launches']})" "$@"; }
for v in base RD0; do
  lib=""; [ "$v" != base ] && lib="build/ablate/libmfg_hip_$v.so"
  MFG_HIP_LIB=$lib timeout -k 10 200 python bench.py --config alltest16.yaml --batch 32768 --steps 200 --warmup 50 --alt-steps 0 --packed-steps 0 --no-cpu-baseline > gpurun_out/c4_$v.json 2>/dev/null || exit 1
  show gpurun_out/c4_$v.json "C4 $v"
done
for v in base R2OFF; do
  lib=""; [ "$v" != base ] && lib="build/ablate/libmfg_hip_$v.so"
  MFG_HIP_LIB=$lib timeout -k 10 400 python bench.py --config grid128_64.yaml --batch 131072 --fuse 1 --steps 10 --warmup 3 --alt-steps 0 --packed-steps 0 --no-cpu-baseline > gpurun_out/c5_$v.json 2>gpurun_out/c5_$v.err || { tail -5 gpurun_out/c5_$v.err; exit 1; }
  show gpurun_out/c5_$v.json "C5 $v"
done
for m in cells segments; do
  MFG_GRU_WINDOW=$m timeout -k 10 300 python tools/bench_marl.py > gpurun_out/marl_$m.json 2>gpurun_out/marl_$m.err || { tail -5 gpurun_out/marl_$m.err; exit 1; }
  echo "$m $(cat gpurun_out/marl_$m.json)"
done
timeout -k 10 300 python bench.py --steps 400 --warmup 100 --alt-steps 0 --packed-steps 0 --no-cpu-baseline > gpurun_out/c3_r03i.json 2>/dev/null || exit 1
show gpurun_out/c3_r03i.json C3

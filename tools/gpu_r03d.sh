#!/bin/bash
# GPU suite (window dirt map parity), C4 with the debt paid every step (RES build), and C2/C4/C5 numbers.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/t_r03d.log 2>&1 || { tail -30 gpurun_out/t_r03d.log; exit 1; }
tail -1 gpurun_out/t_r03d.log
show() { python -c "
import json,sys; d=json.load(open(sys.argv[1]))
print(sys.argv[2], round(d['value']/1e6,4), d['ms_per_step'], {k: (v['launches'], v['mean_launch_ms']) for k, v in d['roofline']['kernels'].items() if v['launches']})" "$@"; }
for v in base RES base RES; do
  lib=""; [ "$v" != base ] && lib="build/ablate/libmfg_hip_$v.so"
  MFG_HIP_LIB=$lib timeout -k 10 200 python bench.py --config alltest16.yaml --batch 32768 --steps 200 --warmup 50 --alt-steps 0 --packed-steps 0 --no-cpu-baseline > gpurun_out/c4_$v.json 2>/dev/null || exit 1
  show gpurun_out/c4_$v.json "C4 $v"
done
timeout -k 10 200 python bench.py --config rooms4.yaml --batch 4096 --steps 400 --warmup 100 --alt-steps 0 --packed-steps 0 --no-cpu-baseline > gpurun_out/c2_r03d.json 2>/dev/null || exit 1
show gpurun_out/c2_r03d.json C2
timeout -k 10 400 python bench.py --config grid128_64.yaml --batch 131072 --fuse 1 --steps 10 --warmup 3 --alt-steps 0 --packed-steps 0 --no-cpu-baseline > gpurun_out/c5_r03d.json 2>gpurun_out/c5_r03d.err || { tail -5 gpurun_out/c5_r03d.err; exit 1; }
show gpurun_out/c5_r03d.json C5

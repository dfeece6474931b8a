#!/bin/bash
# GPU suite (fast SpawnAgents emptiness, per-step replay heuristic), then C4/C2/C3 numbers.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/t_r03e.log 2>&1 || { tail -30 gpurun_out/t_r03e.log; exit 1; }
tail -1 gpurun_out/t_r03e.log
show() { python -c "
import json,sys; d=json.load(open(sys.argv[1]))
print(sys.argv[2], round(d['value']/1e6,4), d['ms_per_step'], {k: (v['launches'], v['mean_launch_ms']) for k, v in d['roofline']['kernels'].items() if v['launches']})" "$@"; }
timeout -k 10 200 python bench.py --config alltest16.yaml --batch 32768 --steps 200 --warmup 50 --alt-steps 0 --packed-steps 0 --no-cpu-baseline > gpurun_out/c4_r03e.json 2>/dev/null || exit 1
show gpurun_out/c4_r03e.json C4
timeout -k 10 200 python bench.py --config rooms4.yaml --batch 4096 --steps 400 --warmup 100 --alt-steps 0 --packed-steps 0 --no-cpu-baseline > gpurun_out/c2_r03e.json 2>/dev/null || exit 1
show gpurun_out/c2_r03e.json C2
timeout -k 10 200 python bench.py --steps 400 --warmup 100 --alt-steps 0 --packed-steps 0 --no-cpu-baseline > gpurun_out/c3_r03e.json 2>/dev/null || exit 1
show gpurun_out/c3_r03e.json C3
timeout -k 10 400 python bench.py --config grid128_64.yaml --batch 131072 --fuse 1 --steps 10 --warmup 3 --alt-steps 0 --packed-steps 0 --no-cpu-baseline > gpurun_out/c5_r03e.json 2>gpurun_out/c5_r03e.err || { tail -5 gpurun_out/c5_r03e.err; exit 1; }
show gpurun_out/c5_r03e.json C5

#!/bin/bash
# Launch-tail probe: k_replay time per env-step at 1x, 2x, 4x the C3 batch and at --fuse 16 (a drain at the end
# of every launch costs a fixed fraction per launch; it shrinks per env when the grid has more rounds).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for cfg in "65536 8" "131072 8" "262144 8" "65536 16"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --batch $1 --fuse $2 --steps 400 --warmup 96 --no-cpu-baseline --alt-steps 0 \
    --packed-steps 0 > gpurun_out/tail_$1_$2.json 2> gpurun_out/tail_$1_$2.err || { tail -5 gpurun_out/tail_$1_$2.err; exit 1; }
  python -c "
import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); k=d['roofline']['kernels']
B=$1; F=$2
print(B, F, round(d['value']/1e6,2), 'replay us/env-step x1e3:', round(k['k_replay']['mean_launch_ms']/(B*F)*1e6,4), {n: v['mean_launch_ms'] for n, v in k.items()})" gpurun_out/tail_$1_$2.json || exit 1
done

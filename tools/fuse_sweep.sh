#!/bin/bash
# fuse length sweep (env-steps per mfg_step call, one k_replay per call)
cd "$GRAFT_REPO_ROOT" || exit 1
for f in 8 16 32; do
  timeout -k 10 300 python bench.py --fuse $f --steps 1024 --warmup 600 --no-cpu-baseline --alt-steps 0 --packed-steps 0 \
    | python -c "
import json,sys; d=json.loads(sys.stdin.readlines()[-1]); k=d['roofline'].get('kernels',{})
print('fuse $f', d['value'], d['ms_per_step'], {n: (v['mean_launch_ms'], v['launches']) for n, v in k.items()})" || exit 1
done

#!/bin/bash
# replay scheduling sweep (timing): debt paid once per K-step call vs every step, and the fuse length
cd "$GRAFT_REPO_ROOT" || exit 1
run() {
  timeout -k 10 300 env "$@" python bench.py --steps 1000 --warmup 600 --no-cpu-baseline --alt-steps 0 --packed-steps 0 \
    | python -c "
import json,sys; d=json.loads(sys.stdin.readlines()[-1]); k=d['roofline'].get('kernels',{})
print('$*', d['value'], d['ms_per_step'], {n: (v['mean_launch_ms'], v['launches']) for n, v in k.items()})"
}
run X=1 && run MFG_REPLAY_EACH_STEP=1

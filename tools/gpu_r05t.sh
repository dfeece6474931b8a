#!/bin/bash
# Round 5: renders with rays of > 12 points back on per-layer stores without the stashed-tag LDS table: GPU suite,
# then C5 / C4 / C2 / C3 lines.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=r05t
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > gpurun_out/${T}_gpu_tests.txt 2>&1 \
  || { tail -30 gpurun_out/${T}_gpu_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_gpu_tests.txt
for c in c5 c4 c2 c3; do
  case $c in
    c2) args="--config rooms4.yaml --batch 4096 --steps 400 --warmup 100";;
    c3) args="--steps 800 --warmup 200";;
    c4) args="--config alltest16.yaml --batch 32768 --steps 100 --warmup 30";;
    c5) args="--config grid128_64.yaml --batch 131072 --fuse 1 --steps 6 --warmup 2";;
  esac
  timeout -k 10 300 python bench.py --no-cpu-baseline --alt-steps 0 --packed-steps 0 $args > gpurun_out/${T}_$c.json 2> gpurun_out/${T}_$c.err || { tail -5 gpurun_out/${T}_$c.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/${T}_$c.json'))
print('$c', round(d['value']/1e6,4), d['ms_per_step'], {k: v.get('mean_launch_ms', v.get('ms_per_step')) for k, v in d['roofline']['kernels'].items()})"
done

#!/bin/bash
# Timing sweep of waves per workgroup for k_logic / k_obs (measurement switches MFG_LOGIC_WPB, MFG_OBS_WPB).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for cfg in "4 4" "1 4" "2 4" "4 1" "4 2"; do
  set -- $cfg
  MFG_LOGIC_WPB=$1 MFG_OBS_WPB=$2 timeout -k 10 200 python bench.py --no-cpu-baseline --alt-steps 0 --packed-steps 0 \
    --steps 800 --warmup 200 > gpurun_out/wpb_$1_$2.json 2>/dev/null || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/wpb_$1_$2.json'))
print('logic_wpb $1 obs_wpb $2', round(d['value']/1e6,2), {k: v['mean_launch_ms'] for k, v in d['roofline']['kernels'].items()})"
done

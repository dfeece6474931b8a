#!/bin/bash
# A/B timing: the previous build (build/ablate/libmfg_hip_R02G.so), the in-tree build, and the in-tree build with
# the env switches given as arguments (e.g. MFG_REPLAY_LPT=1), alternating, 2 rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for r in 1 2; do
  for v in prev cur "$@"; do
    lib=""; envs=""
    [ "$v" = prev ] && lib="build/ablate/libmfg_hip_R02G.so"
    [ "$v" != prev ] && [ "$v" != cur ] && envs="$v"
    env MFG_HIP_LIB=$lib $envs timeout -k 10 200 python bench.py --no-cpu-baseline --alt-steps 0 --packed-steps 0 \
      --steps 800 --warmup 200 > gpurun_out/ab_$r.json 2>gpurun_out/ab_$r.err || { tail -5 gpurun_out/ab_$r.err; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/ab_$r.json').read().strip().splitlines()[-1])
print('$v', round(d['value']/1e6,3), {k: v['mean_launch_ms'] for k, v in d['roofline']['kernels'].items()})" || exit 1
  done
done

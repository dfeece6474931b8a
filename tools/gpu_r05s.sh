#!/bin/bash
# Round 5: C5's render unit (18-point rays, k_obs_mw) with the flattened stores (in-tree) vs per-layer stores (NOFLATC).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=r05s
for r in 1 2; do
  for v in base NOFLATC; do
    lib=""; [ "$v" != base ] && lib="build/ablate/libmfg_hip_$v.so"
    MFG_HIP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --alt-steps 0 --packed-steps 0 --config grid128_64.yaml --batch 131072 --fuse 1 --steps 6 --warmup 2 > gpurun_out/${T}_c5_$v.json 2> gpurun_out/${T}_c5_$v.err || { tail -5 gpurun_out/${T}_c5_$v.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/${T}_c5_$v.json'))
print('c5 $v', round(d['value']/1e6,4), d['ms_per_step'], {k: v.get('mean_launch_ms', v.get('ms_per_step')) for k, v in d['roofline']['kernels'].items()})"
  done
done

#!/bin/bash
# Round 5: C4's multi-wave render with the flattened stores non-temporal (C4NT: -DMFG_OBS_PLAIN_PTS=0 in unit b) vs
# plain (in-tree), overlapped and serial lines.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=r05ac
for r in 1 2; do
  for v in base C4NT; do
    lib=""; [ "$v" != base ] && lib="build/ablate/libmfg_hip_$v.so"
    for s in "" "--serial"; do
      MFG_HIP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --alt-steps 0 --packed-steps 0 --config alltest16.yaml --batch 32768 --steps 100 --warmup 30 $s > gpurun_out/${T}_c4_$v$s.json 2> gpurun_out/${T}_c4_$v.err || { tail -5 gpurun_out/${T}_c4_$v.err; exit 1; }
      python -c "
import json; d=json.load(open('gpurun_out/${T}_c4_$v$s.json'))
print('c4 $v $s', d['value'], d['ms_per_step'], {k: v.get('mean_launch_ms', v.get('ms_per_step')) for k, v in d['roofline']['kernels'].items()})"
    done
  done
done

#!/bin/bash
# Round 5: C4 with the second stream (resets + per-step replay) at the lowest priority (PLO) vs the highest (in-tree).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=r05aj
python -c "import torch; print('priority range', torch.cuda.Stream.priority_range())" || true
for r in 1 2; do
  for v in base PLO; do
    lib=""; [ "$v" != base ] && lib="build/ablate/libmfg_hip_$v.so"
    MFG_HIP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --alt-steps 0 --packed-steps 0 --config alltest16.yaml --batch 32768 --steps 200 --warmup 50 > gpurun_out/${T}_c4_$v.json 2> gpurun_out/${T}_c4_$v.err || { tail -5 gpurun_out/${T}_c4_$v.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/${T}_c4_$v.json'))
print('c4 $v', d['value'], d['ms_per_step'], {k: v.get('mean_launch_ms', v.get('ms_per_step')) for k, v in d['roofline']['kernels'].items()})"
  done
done

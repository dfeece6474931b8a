#!/bin/bash
# Round 5: C3 render ablations (no flattened pass / no stores) and branch-free special layer values (SEL): parity of
# SEL on the render tests, then the C3 A/B and C4.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=r05ah
MFG_HIP_LIB=build/ablate/libmfg_hip_SEL.so timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_marl.py -k "large8 or rooms4 or alltest16 or simple1 or obs_test or packed" > gpurun_out/${T}_tests.txt 2>&1 \
  || { tail -30 gpurun_out/${T}_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_tests.txt
bash tools/ab_run.sh SEL || exit 1
for v in base SEL; do
  lib=""; [ "$v" != base ] && lib="build/ablate/libmfg_hip_$v.so"
  MFG_HIP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --alt-steps 0 --packed-steps 0 --config alltest16.yaml --batch 32768 --steps 200 --warmup 50 > gpurun_out/${T}_c4_$v.json 2> gpurun_out/${T}_c4_$v.err || { tail -5 gpurun_out/${T}_c4_$v.err; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/${T}_c4_$v.json'))
print('c4 $v', d['value'], d['ms_per_step'], {k: v.get('mean_launch_ms', v.get('ms_per_step')) for k, v in d['roofline']['kernels'].items()})"
done

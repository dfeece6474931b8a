#!/bin/bash
# Round 5: C4's per-step replay on the caller's stream after the render (RMAIN: -DMFG_REPLAY_MAIN=1) vs on the
# second stream beside it (in-tree): parity of RMAIN on the split-mode tests, then C4 A/B.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=r05af
MFG_HIP_LIB=build/ablate/libmfg_hip_RMAIN.so timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_timed_path.py -k "alltest16 or serial or pair_spill or fused or deferred" > gpurun_out/${T}_tests.txt 2>&1 \
  || { tail -30 gpurun_out/${T}_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_tests.txt
for r in 1 2; do
  for v in base RMAIN; do
    lib=""; [ "$v" != base ] && lib="build/ablate/libmfg_hip_$v.so"
    MFG_HIP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --alt-steps 0 --packed-steps 0 --config alltest16.yaml --batch 32768 --steps 200 --warmup 50 > gpurun_out/${T}_c4_$v.json 2> gpurun_out/${T}_c4_$v.err || { tail -5 gpurun_out/${T}_c4_$v.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/${T}_c4_$v.json'))
print('c4 $v', d['value'], d['ms_per_step'], {k: v.get('mean_launch_ms', v.get('ms_per_step')) for k, v in d['roofline']['kernels'].items()})"
  done
done

#!/bin/bash
# env_reset inlined (k_resetdone at 4 waves/SIMD) + k_replay_done work queue: GPU suite, C3 and C4 A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/t_r03m.log 2>&1 || { tail -30 gpurun_out/t_r03m.log; exit 1; }
tail -1 gpurun_out/t_r03m.log
./tools/ab_run.sh INL0 RPDQ0 || exit 1
for v in base INL0; do
  lib=""; [ "$v" != base ] && lib="build/ablate/libmfg_hip_$v.so"
  MFG_HIP_LIB=$lib timeout -k 10 200 python bench.py --config alltest16.yaml --batch 32768 --steps 200 --warmup 50 --alt-steps 0 --packed-steps 0 --no-cpu-baseline > gpurun_out/c4_$v.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/c4_$v.json')); k=d['roofline']['kernels']; print('C4 $v', d['value'], d['ms_per_step'], k['k_resetdone']['mean_launch_ms'], k.get('resets_exposed'))"
done
echo done

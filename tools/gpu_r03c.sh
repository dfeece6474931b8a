#!/bin/bash
# GPU suite on the current build (RPV3 swap blocks, reset overlap heuristic, k_replay_sel), then A/B of the
# overlap on C3 (heuristic: off) and C4 (heuristic: on).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/t_r03c.log 2>&1 || { tail -30 gpurun_out/t_r03c.log; exit 1; }
tail -1 gpurun_out/t_r03c.log
./tools/ab_run.sh OVL2 || exit 1
for r in 1 2; do
for v in base OVL0; do
  lib=""; [ "$v" != base ] && lib="build/ablate/libmfg_hip_$v.so"
  MFG_HIP_LIB=$lib timeout -k 10 200 python bench.py --config alltest16.yaml --batch 32768 --steps 200 --warmup 50 --alt-steps 0 --packed-steps 0 --no-cpu-baseline > gpurun_out/c4_$v.json 2>/dev/null || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/c4_$v.json'))
print('C4 $v', round(d['value']/1e6,3), d['ms_per_step'], {k: (v['launches'], v['mean_launch_ms']) for k, v in d['roofline']['kernels'].items()})"
done
done

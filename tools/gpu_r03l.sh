#!/bin/bash
# Door points from the ray registers (MFG_DYN_REG): GPU suite, A/B against the table reload, k_obs phase ablations.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/t_r03l.log 2>&1 || { tail -30 gpurun_out/t_r03l.log; exit 1; }
tail -1 gpurun_out/t_r03l.log
./tools/ab_run.sh DYN0 OB_NORAY OB_NODEDUP OB_NOPLACE OB_NOSTORE || exit 1
for v in base DYN0; do
  lib=""; [ "$v" != base ] && lib="build/ablate/libmfg_hip_$v.so"
  MFG_HIP_LIB=$lib timeout -k 10 200 python bench.py --config alltest16.yaml --batch 32768 --steps 200 --warmup 50 --alt-steps 0 --packed-steps 0 --no-cpu-baseline > gpurun_out/c4_$v.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/c4_$v.json')); print('C4 $v', d['value'], d['ms_per_step'], d['roofline']['kernels']['k_obs']['mean_launch_ms'])"
done
echo done

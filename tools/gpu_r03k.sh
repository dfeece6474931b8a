#!/bin/bash
# Packed entries-only render + whole-wave table clears: parity (packed + timed path), A/B of the clears, packed lines.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_marl.py tests/test_gpu_timed_path.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/t_r03k.log 2>&1 || { tail -30 gpurun_out/t_r03k.log; exit 1; }
tail -1 gpurun_out/t_r03k.log
./tools/ab_run.sh FILL0 || exit 1
for v in base PK1H0; do
  lib=""; [ "$v" != base ] && lib="build/ablate/libmfg_hip_$v.so"
  MFG_HIP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --alt-steps 0 --steps 800 --warmup 200 > gpurun_out/pk_$v.json 2>/dev/null || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/pk_$v.json')); p=d['packed_obs']
print('$v dense', d['value'], 'packed', p['value'], p['ms_per_step'], 'fused', p['fused_proj']['value'], 'dense+proj', p['dense_f32_plus_proj']['value'])"
done
echo done

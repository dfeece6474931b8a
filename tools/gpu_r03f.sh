#!/bin/bash
# Packed-obs parity (test_marl) + the default bench line (dense f32, f64 and packed lines).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_marl.py tests/test_gpu_timed_path.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/t_r03f.log 2>&1 || { tail -30 gpurun_out/t_r03f.log; exit 1; }
tail -1 gpurun_out/t_r03f.log
timeout -k 10 400 python bench.py --steps 400 --warmup 100 --no-cpu-baseline > gpurun_out/b_r03f.json 2>gpurun_out/b_r03f.err || { tail -5 gpurun_out/b_r03f.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/b_r03f.json'))
print('dense', d['value'], 'f64', d['alt_obs_dtype']['value'], 'packed', d['packed_obs']['value'], d['packed_obs']['ms_per_step'])
print({k: v['mean_launch_ms'] for k, v in d['roofline']['kernels'].items()})"

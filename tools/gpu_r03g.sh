#!/bin/bash
# Packed-obs parity after the queued stores; bench (dense / f64 / packed / dense+proj); A2C loop throughput.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/t_r03g.log 2>&1 || { tail -30 gpurun_out/t_r03g.log; exit 1; }
tail -1 gpurun_out/t_r03g.log
timeout -k 10 400 python bench.py --steps 400 --warmup 100 --no-cpu-baseline > gpurun_out/b_r03g.json 2>gpurun_out/b_r03g.err || { tail -5 gpurun_out/b_r03g.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/b_r03g.json'))
p=d['packed_obs']
print('dense', d['value'], 'f64', d['alt_obs_dtype']['value'], 'packed', p['value'], p['ms_per_step'], 'dense+proj', p['dense_f32_plus_proj'])"
timeout -k 10 300 python tools/bench_marl.py > gpurun_out/marl_r03g.json 2>gpurun_out/marl_r03g.err || { tail -5 gpurun_out/marl_r03g.err; exit 1; }
cat gpurun_out/marl_r03g.json

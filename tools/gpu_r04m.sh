#!/bin/bash
# Default bench line (f64 headline + side lines + CPU baseline), then rocprofv3 kernel stats of the same command.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python bench.py > gpurun_out/r04m_bench.json 2> gpurun_out/r04m_bench.err || { tail -20 gpurun_out/r04m_bench.err; exit 1; }
python - <<'PY'
import json
d = json.load(open('gpurun_out/r04m_bench.json'))
r = d['roofline']
print('value', d['value'], d['ms_per_step'], d['dtype'], 'frac', r['frac'], 'sec8d', r.get('frac_sec8d'))
print({k: round(v['mean_launch_ms'], 4) for k, v in r['kernels'].items() if 'mean_launch_ms' in v})
print('alt', d.get('alt_obs_dtype', {}) and {k: d['alt_obs_dtype'][k] for k in ('obs', 'value', 'ms_per_step')})
p = d.get('packed_obs') or {}
print('packed', p.get('value'), 'fused', (p.get('fused_proj') or {}).get('value'), 'dense+proj', (p.get('dense_f32_plus_proj') or {}).get('value'))
print('cpu', d.get('cpu_baseline'))
PY
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r04m_prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/r04m_prof.log 2>&1 || { tail -5 gpurun_out/r04m_prof.log; exit 1; }
echo prof ok

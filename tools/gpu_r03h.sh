#!/bin/bash
# Full GPU suite (two-wave replay on the grid128 configs, relaxed obs limits, queued packed stores, GRU windows),
# the two-wave replay forced on the C3/C2 parity cases, bench (dense/f64/packed/dense+proj), A2C loop, C5.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/t_r03h.log 2>&1 || { tail -30 gpurun_out/t_r03h.log; exit 1; }
tail -1 gpurun_out/t_r03h.log
MFG_HIP_LIB=build/ablate/libmfg_hip_RP2F.so timeout -k 10 600 python -u -m pytest tests/test_gpu_timed_path.py tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread -k "timed_path_k8 or large8 or rooms4 or alltest16" > gpurun_out/t_r03h_rp2.log 2>&1 || { tail -30 gpurun_out/t_r03h_rp2.log; exit 1; }
tail -1 gpurun_out/t_r03h_rp2.log
timeout -k 10 400 python bench.py --steps 400 --warmup 100 --no-cpu-baseline > gpurun_out/b_r03h.json 2>gpurun_out/b_r03h.err || { tail -5 gpurun_out/b_r03h.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/b_r03h.json'))
p=d['packed_obs']
print('dense', d['value'], 'f64', d['alt_obs_dtype']['value'], 'packed', p['value'], p['ms_per_step'], 'dense+proj', p['dense_f32_plus_proj'])"
timeout -k 10 300 python tools/bench_marl.py > gpurun_out/marl_r03h.json 2>gpurun_out/marl_r03h.err || { tail -5 gpurun_out/marl_r03h.err; exit 1; }
cat gpurun_out/marl_r03h.json
timeout -k 10 400 python bench.py --config grid128_64.yaml --batch 131072 --fuse 1 --steps 10 --warmup 3 --alt-steps 0 --packed-steps 0 --no-cpu-baseline > gpurun_out/c5_r03h.json 2>gpurun_out/c5_r03h.err || { tail -5 gpurun_out/c5_r03h.err; exit 1; }
python -c "
import json,sys; d=json.load(open('gpurun_out/c5_r03h.json'))
print('C5', d['value'], d['ms_per_step'], {k: (v['launches'], v['mean_launch_ms']) for k, v in d['roofline']['kernels'].items() if v['launches']})"
./tools/ab_run.sh NOCLAMP || exit 1
for v in base PKW1; do
  lib=""; [ "$v" != base ] && lib="build/ablate/libmfg_hip_$v.so"
  MFG_HIP_LIB=$lib timeout -k 10 300 python bench.py --steps 400 --warmup 100 --alt-steps 0 --no-cpu-baseline > gpurun_out/pk_$v.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/pk_$v.json')); print('$v packed', d['packed_obs']['value'], d['packed_obs']['ms_per_step'], 'dense', d['value'])"
done

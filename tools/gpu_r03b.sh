#!/bin/bash
# Reset/render overlap parity check, LDS probe v2, k_replay swap-block variants A/B (+ no-overlap build), C4 A/B,
# LDS PMC per variant.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_timed_path.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_r03b.log 2>&1 || { tail -30 gpurun_out/t_r03b.log; exit 1; }
tail -1 gpurun_out/t_r03b.log
timeout -k 10 120 ./build/lds_probe > gpurun_out/lds_probe2.txt 2>&1 || { cat gpurun_out/lds_probe2.txt; exit 1; }
cat gpurun_out/lds_probe2.txt
./tools/ab_run.sh NOOVL RPV3 RPV7 RPV11 || exit 1
for v in base NOOVL; do
  lib=""; [ "$v" != base ] && lib="build/ablate/libmfg_hip_$v.so"
  MFG_HIP_LIB=$lib timeout -k 10 200 python bench.py --config alltest16.yaml --batch 32768 --steps 200 --warmup 50 --alt-steps 0 --packed-steps 0 --no-cpu-baseline > gpurun_out/c4_$v.json 2>/dev/null || exit 1
  python -c "
import json; d=json.load(open('gpurun_out/c4_$v.json'))
print('C4 $v', round(d['value']/1e6,3), d['ms_per_step'], {k: (v['launches'], v['mean_launch_ms']) for k, v in d['roofline']['kernels'].items()})"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in base RPV3 RPV7 RPV11; do
  lib=""; [ "$v" != base ] && lib="build/ablate/libmfg_hip_$v.so"
  MFG_HIP_LIB=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_SALU -d gpurun_out/pmcl_$v -o run --output-format csv -- python3 bench.py --steps 16 --warmup 8 --no-cpu-baseline --no-profile --alt-steps 0 --packed-steps 0 > gpurun_out/pmcl_$v.log 2>&1 || { tail -5 gpurun_out/pmcl_$v.log; exit 1; }
  python3 - "$v" <<'PY'
import csv, glob, sys
v = sys.argv[1]
f = glob.glob(f'gpurun_out/pmcl_{v}/**/*counter_collection.csv', recursive=True)[0]
acc = {}
for r in csv.DictReader(open(f)):
    if not r['Kernel_Name'].startswith('k_replay('):
        continue
    acc.setdefault(r['Counter_Name'], []).append(float(r['Counter_Value']))
print(v, {k: round(sum(x) / len(x) / 1e9, 4) for k, x in acc.items()}, 'x1e9 per dispatch (n=%d)' % len(next(iter(acc.values()))))
PY
done

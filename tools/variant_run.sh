#!/bin/bash
# Run on the GPU box: time the in-tree engine (BASE) and each build/var variant on the C3 bench, and
# run the quick parity subset against each variant. usage: tools/variant_run.sh [--parity] NAME ...
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
PAR=0; if [ "$1" = --parity ]; then PAR=1; shift; fi
for v in BASE "$@"; do
  if [ $v = BASE ]; then unset MFG_HIP_LIB; else export MFG_HIP_LIB=$PWD/build/var/libmfg_hip_$v.so; fi
  if [ $PAR = 1 ] && [ $v != BASE ]; then
    timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -x -q -k "large8 or rooms4 or grid128" > gpurun_out/vpar_$v.log 2>&1 || { echo "$v parity FAILED"; tail -20 gpurun_out/vpar_$v.log; exit 1; }
    echo "$v parity: $(tail -1 gpurun_out/vpar_$v.log)"
  fi
  timeout -k 10 300 python bench.py --steps 400 --warmup 100 --no-cpu-baseline "${BENCH_ARGS[@]}" > gpurun_out/var_$v.json 2> gpurun_out/var_$v.err || { tail -5 gpurun_out/var_$v.err; exit 1; }
  python -c "
import json,sys; d=json.loads(open(sys.argv[1]).readlines()[-1]); k=d['roofline'].get('kernels',{})
print('$v', d['value'], d['ms_per_step'], {n: v['mean_launch_ms'] for n, v in k.items()})" gpurun_out/var_$v.json || exit 1
done

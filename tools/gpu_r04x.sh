#!/bin/bash
# Two-wave replay with the producer's MT in the record (GMT variant, 5 envs per CU at C5): grid128 parity with the
# variant and with the in-tree library, then C5 A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in GMT base; do
  lib=""; [ $v = GMT ] && lib=build/ablate/libmfg_hip_GMT.so
  MFG_HIP_LIB=$lib timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_parity.py \
    -k "grid128 or qquad" > gpurun_out/r04x_tests_$v.txt 2>&1 || { tail -30 gpurun_out/r04x_tests_$v.txt; exit 1; }
  echo "$v: $(tail -1 gpurun_out/r04x_tests_$v.txt)"
done
for v in base GMT; do
  lib=""; [ $v = GMT ] && lib=build/ablate/libmfg_hip_GMT.so
  MFG_HIP_LIB=$lib timeout -k 10 500 python bench.py --no-cpu-baseline --alt-steps 0 --packed-steps 0 --config grid128_64.yaml \
    --batch 131072 --fuse 1 --steps 6 --warmup 3 > gpurun_out/r04x_c5_$v.json 2> gpurun_out/r04x_c5_$v.err || { tail -5 gpurun_out/r04x_c5_$v.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['roofline']['kernels']; print(sys.argv[2], round(d['value']), round(d['ms_per_step'],2), {n: round(x['mean_launch_ms'],2) for n,x in k.items() if 'mean_launch_ms' in x})" gpurun_out/r04x_c5_$v.json $v
done

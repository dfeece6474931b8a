#!/bin/bash
# Per-step replay beside the render (C4): K=8 vs K=1 equality + alltest16 parity, then C4 A/B vs the previous library.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_timed_path.py tests/test_gpu_parity.py \
  -k "fused_k8 or alltest16 or output_rows" > gpurun_out/r04w_tests.txt 2>&1 || { tail -30 gpurun_out/r04w_tests.txt; exit 1; }
tail -1 gpurun_out/r04w_tests.txt
for r in 1 2; do
for v in OLD new; do
  lib=""; [ $v = OLD ] && lib=build/ablate/libmfg_hip_OLD.so
  MFG_HIP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --alt-steps 0 --packed-steps 0 --config alltest16.yaml \
    --batch 32768 --steps 200 --warmup 50 > gpurun_out/r04w_c4_${v}_$r.json 2> gpurun_out/r04w_c4_${v}_$r.err || { tail -5 gpurun_out/r04w_c4_${v}_$r.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['roofline']['kernels']; print(sys.argv[2], round(d['value']), round(d['ms_per_step'],4), {n: round(x['mean_launch_ms'],3) for n,x in k.items() if 'mean_launch_ms' in x})" gpurun_out/r04w_c4_${v}_$r.json $v
done
done

#!/bin/bash
# k_logic with maintainers split (lean + maintainer staging where no maintainer re-routes): maintainer parity tests,
# then C5 A/B against the previous library (build/ablate/libmfg_hip_OLD.so).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_parity.py tests/test_facade.py tests/test_gpu_timed_path.py \
  -k "grid128 or maint or alltest16 or bfs" > gpurun_out/r04u_tests.txt 2>&1 || { tail -30 gpurun_out/r04u_tests.txt; exit 1; }
tail -1 gpurun_out/r04u_tests.txt
for v in OLD new; do
  lib=""; [ $v = OLD ] && lib=build/ablate/libmfg_hip_OLD.so
  MFG_HIP_LIB=$lib timeout -k 10 500 python bench.py --no-cpu-baseline --alt-steps 0 --packed-steps 0 --config grid128_64.yaml \
    --batch 131072 --fuse 1 --steps 6 --warmup 3 > gpurun_out/r04u_c5_$v.json 2> gpurun_out/r04u_c5_$v.err || { tail -5 gpurun_out/r04u_c5_$v.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['roofline']['kernels']; print(sys.argv[2], round(d['value']), round(d['ms_per_step'],2), {n: round(x['mean_launch_ms'],2) for n,x in k.items() if 'mean_launch_ms' in x})" gpurun_out/r04u_c5_$v.json $v
done

#!/bin/bash
# Round-4 GPU tests of the new paths (multi-rank engine processes, f64 timed mode, 48/64-point rays, variant-forced
# paths), the 2-rank shared-GPU bench and the A2C loop.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_ranks.py tests/test_gpu_timed_path.py tests/test_gpu_parity.py tests/test_marl.py \
  -m gpu -v --timeout 800 --timeout-method thread > gpurun_out/r04b_tests.log 2>&1 || { tail -40 gpurun_out/r04b_tests.log; exit 1; }
tail -3 gpurun_out/r04b_tests.log
MFG_BENCH_SHARE_GPU=1 timeout -k 10 400 python bench.py --gpus 2 --backend gloo --warmup 600 --steps 400 \
  --alt-steps 0 --packed-steps 0 > gpurun_out/r04b_share2_bench.json 2> gpurun_out/r04b_share2_bench.err \
  || { tail -20 gpurun_out/r04b_share2_bench.err; exit 1; }
head -c 600 gpurun_out/r04b_share2_bench.json
echo
timeout -k 10 300 python tools/bench_marl.py --updates 20 > gpurun_out/r04b_marl.json 2> gpurun_out/r04b_marl.err \
  || { tail -20 gpurun_out/r04b_marl.err; exit 1; }
cat gpurun_out/r04b_marl.json

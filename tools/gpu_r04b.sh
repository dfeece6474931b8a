#!/bin/bash
# Round-4 k_replay attribution + first variants: CPU share probe, ablations and exact variants A/B against the in-tree
# library, then the new GPU tests (multi-rank, f64 timed path, long-ray fixtures) and the 2-rank shared-GPU bench.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
{ echo "cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)"; echo "nproc: $(nproc)";
  python -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())"; } > gpurun_out/r04b_cpu.txt 2>&1
cat gpurun_out/r04b_cpu.txt
timeout -k 10 200 python tools/cpu_sweep.py 4 1 8 16 32 64 128 > gpurun_out/r04b_cpu_sweep.json || exit 1
bash tools/ab_run.sh SINK0 YWC1 IW1 NODEBT NOSWAP NOSWAPTW NOTWIST NOFWD NOJAC || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_ranks.py tests/test_gpu_timed_path.py tests/test_gpu_parity.py \
  -m gpu -v --timeout 800 --timeout-method thread > gpurun_out/r04b_tests.log 2>&1 || { tail -40 gpurun_out/r04b_tests.log; exit 1; }
tail -3 gpurun_out/r04b_tests.log
MFG_BENCH_SHARE_GPU=1 timeout -k 10 400 python bench.py --gpus 2 --backend gloo --warmup 600 --steps 400 \
  --alt-steps 0 --packed-steps 0 > gpurun_out/r04b_share2_bench.json 2> gpurun_out/r04b_share2_bench.err \
  || { tail -20 gpurun_out/r04b_share2_bench.err; exit 1; }
head -c 600 gpurun_out/r04b_share2_bench.json

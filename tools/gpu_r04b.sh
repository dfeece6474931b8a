#!/bin/bash
# Round-4 k_replay attribution + first variants: CPU share probe, ablations and exact variants A/B against the in-tree
# library, then the new GPU tests (multi-rank, f64 timed path, long-ray fixtures) and the 2-rank shared-GPU bench.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
{ echo "cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)"; echo "nproc: $(nproc)";
  python -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())"; } > gpurun_out/r04b_cpu.txt 2>&1
cat gpurun_out/r04b_cpu.txt
timeout -k 10 200 python tools/cpu_sweep.py 4 1 8 16 32 64 128 > gpurun_out/r04b_cpu_sweep.json || exit 1
bash tools/ab_run.sh SINK0 YWC1 IW1 NT64_0 NODEBT NOSWAP NOSWAPTW NOTWIST NOFWD NOJAC || exit 1

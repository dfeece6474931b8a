#!/bin/bash
# Round-4 k_replay attribution: the box's CPU share, then timing-only ablation builds against the in-tree library.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
{ echo "cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>/dev/null)"; echo "nproc: $(nproc)";
  python -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())"; } > gpurun_out/r04a_cpu.txt 2>&1
cat gpurun_out/r04a_cpu.txt
timeout -k 10 200 python tools/cpu_sweep.py 4 1 8 16 32 64 128 > gpurun_out/r04a_cpu_sweep.json || exit 1
bash tools/ab_run.sh NODEBT NOSWAP NOSWAPTW NOTWIST NOFWD NOJAC

#!/bin/bash
# Round 5: replay tail chunks with per-rank widths (RP_TAIL 62, in-tree) vs band-only chunks (T0: RP_TAIL -1): the
# GPU suite first (every shuffle and reset draw goes through it), then the fixed replay workload and the bench A/B.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=r05n
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > gpurun_out/${T}_gpu_tests.txt 2>&1 \
  || { tail -30 gpurun_out/${T}_gpu_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_gpu_tests.txt
bash tools/replay_ab.sh T0 || exit 1
bash tools/ab_run.sh T0 || exit 1

#!/bin/bash
# Round 5: kernels of the A2C acting step (torch profiler), and the C3 render's store cost with the flattened stores.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python tools/prof_a2c_act.py > gpurun_out/r05l_prof_act.txt 2>&1 || { tail -10 gpurun_out/r05l_prof_act.txt; exit 1; }
head -50 gpurun_out/r05l_prof_act.txt | cut -c1-200
bash tools/ab_run.sh ONOSTORE || exit 1

#!/bin/bash
# GPU-box check: parity tests, a short bench, and a rocprofv3 kernel-trace summary (run via gpurun).
# usage: tools/gpu_round.sh TAG [bench args...]
TAG=${1:-x}; shift
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_parity.py -x -q > gpurun_out/t_$TAG.log 2>&1 || { tail -30 gpurun_out/t_$TAG.log; exit 1; }
tail -2 gpurun_out/t_$TAG.log
timeout -k 10 300 python bench.py --steps 48 --warmup 16 --no-cpu-baseline "$@" > gpurun_out/b_$TAG.log 2>&1 || { tail -20 gpurun_out/b_$TAG.log; exit 1; }
tail -1 gpurun_out/b_$TAG.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --steps 24 --warmup 8 --no-cpu-baseline "$@" > gpurun_out/prof_$TAG.log 2>&1 || { tail -20 gpurun_out/prof_$TAG.log; exit 1; }
find gpurun_out/prof_$TAG -name '*kernel_stats.csv' -exec cat {} \;

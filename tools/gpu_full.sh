#!/bin/bash
# Round-end evidence on the GPU box: parity tests, smoke, the default bench line, a rocprofv3
# kernel-trace summary of the same workload, and the PMC passes. usage: tools/gpu_full.sh TAG
TAG=${1:-x}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/t_$TAG.log 2>&1 || { tail -30 gpurun_out/t_$TAG.log; exit 1; }
tail -1 gpurun_out/t_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || { tail -20 gpurun_out/prof_$TAG.log; exit 1; }
find gpurun_out/prof_$TAG -name '*kernel_stats.csv' -exec cat {} \;
./tools/pmc_run.sh $TAG

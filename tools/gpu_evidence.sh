#!/bin/bash
# GPU evidence, part 1: the whole -m gpu suite, smoke, and the default bench line.
# usage: tools/gpu_evidence.sh TAG   -> gpurun_out/{t,smoke,bench}_TAG.*
TAG=${1:-x}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "gpurun_out/t_$TAG.log" 2>&1 || { tail -30 "gpurun_out/t_$TAG.log"; exit 1; }
tail -2 "gpurun_out/t_$TAG.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "gpurun_out/smoke_$TAG.log" 2>&1 || { tail -20 "gpurun_out/smoke_$TAG.log"; exit 1; }
tail -1 "gpurun_out/smoke_$TAG.log"
timeout -k 10 400 python bench.py > "gpurun_out/bench_$TAG.json" 2> "gpurun_out/bench_$TAG.err" || { tail -20 "gpurun_out/bench_$TAG.err"; exit 1; }
cat "gpurun_out/bench_$TAG.json"

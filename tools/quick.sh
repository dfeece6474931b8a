#!/bin/bash
# Quick GPU iteration: full parity suite, then a short C3 bench line. usage: tools/quick.sh TAG [bench args]
TAG=${1:-x}; shift
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/q_$TAG.log 2>&1 || { tail -30 gpurun_out/q_$TAG.log; exit 1; }
tail -1 gpurun_out/q_$TAG.log
timeout -k 10 300 python bench.py --steps 800 --warmup 200 --no-cpu-baseline "$@" > gpurun_out/qb_$TAG.json 2> gpurun_out/qb_$TAG.err || { tail -5 gpurun_out/qb_$TAG.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['roofline']['kernels']; print(d['value'], d['ms_per_step'], {n: v['mean_launch_ms'] for n, v in k.items()})" gpurun_out/qb_$TAG.json

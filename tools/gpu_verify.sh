#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/t_${TAG:-r03e}.log 2>&1 || { tail -30 gpurun_out/t_${TAG:-r03e}.log; exit 1; }
tail -1 gpurun_out/t_${TAG:-r03e}.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_${TAG:-r03e}.log 2>&1 || { tail -20 gpurun_out/smoke_${TAG:-r03e}.log; exit 1; }
tail -1 gpurun_out/smoke_${TAG:-r03e}.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_${TAG:-r03e}.json 2> gpurun_out/bench_${TAG:-r03e}.err || { tail -20 gpurun_out/bench_${TAG:-r03e}.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_${TAG:-r03e}.json')); print(d['value'], d['ms_per_step'], d['roofline']['mean_launch_ms'])"

#!/bin/bash
# Round-3 first GPU call: LDS pattern probe, the -m gpu suite, the driver's bench form, and the --gpus 2 refusal.
TAG=${1:-r03a}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 ./build/lds_probe > gpurun_out/lds_probe_$TAG.txt 2>&1 || { cat gpurun_out/lds_probe_$TAG.txt; exit 1; }
cat gpurun_out/lds_probe_$TAG.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_$TAG.log 2>&1 || { tail -30 gpurun_out/t_$TAG.log; exit 1; }
tail -2 gpurun_out/t_$TAG.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_$TAG.json')); print(d['value'], d['n_ranks_rccl'], {k:(v['unit'],v['frac']) for k,v in d['roofline']['issue'].items()})"
timeout -k 10 120 python bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/bench2_$TAG.json 2> gpurun_out/bench2_$TAG.err; echo "gpus2 rc=$?"; tail -2 gpurun_out/bench2_$TAG.err

#!/bin/bash
# Round 5: lean maintainer steps write back only the maintainer states (paths read-only there); A2C bookkeeping per
# window. GPU suite, the C5 line and its per-launch k_logic FETCH/WRITE passes.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=r05ab
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > gpurun_out/${T}_gpu_tests.txt 2>&1 \
  || { tail -30 gpurun_out/${T}_gpu_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_gpu_tests.txt
timeout -k 10 300 python bench.py --no-cpu-baseline --alt-steps 0 --packed-steps 0 --config grid128_64.yaml --batch 131072 --fuse 1 --steps 6 --warmup 2 > gpurun_out/${T}_c5.json 2> gpurun_out/${T}_c5.err || { tail -5 gpurun_out/${T}_c5.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/${T}_c5.json'))
print('c5', d['value'], d['ms_per_step'], {k: v.get('mean_launch_ms', v.get('ms_per_step')) for k, v in d['roofline']['kernels'].items()})"
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-profile --alt-steps 0 --packed-steps 0 --config grid128_64.yaml --batch 131072 --fuse 1"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmc_${T}_c5_fetch -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc_${T}_c5_fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/pmc_${T}_c5_write -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc_${T}_c5_write.log 2>&1 || exit 1
echo pmc done
timeout -k 10 300 python tools/bench_marl.py > gpurun_out/${T}_marl.json 2> gpurun_out/${T}_marl.err || { tail -5 gpurun_out/${T}_marl.err; exit 1; }
cat gpurun_out/${T}_marl.json

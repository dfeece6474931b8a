#!/bin/bash
# Round-end evidence on the final tree. Part A: the GPU suite, smoke, the default bench line.
# Part B: rocprofv3 kernel statistics of the bench, the PMC passes (tools/pmc_run.sh), the per-config lines.
# usage (GPU box via gpurun): tools/gpu_final.sh A|B TAG
PART=${1:-A}; T=${2:-r06f}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ "$PART" = A ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.txt 2>&1 \
    || { tail -30 gpurun_out/${T}_gpu_tests.txt; exit 1; }
  tail -1 gpurun_out/${T}_gpu_tests.txt
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1 || { tail -20 gpurun_out/${T}_smoke.txt; exit 1; }
  tail -2 gpurun_out/${T}_smoke.txt
  timeout -k 10 400 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/${T}_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d['cpu_baseline'])"
else
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python3 bench.py --no-cpu-baseline --steps 200 --warmup 50 > gpurun_out/${T}_prof.log 2>&1 \
    || { tail -20 gpurun_out/${T}_prof.log; exit 1; }
  bash tools/pmc_run.sh ${T} > gpurun_out/${T}_pmc.log 2>&1 || { tail -20 gpurun_out/${T}_pmc.log; exit 1; }
  tail -1 gpurun_out/${T}_pmc.log
  bash tools/bench_configs.sh ${T} || exit 1
fi

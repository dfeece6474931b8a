#!/bin/bash
# Round-5 evidence on the final tree: GPU suite, smoke, default bench line, rocprof kernel stats of the same
# command, A2C throughput.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r05z}
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > gpurun_out/${T}_gpu_tests.txt 2>&1 \
  || { tail -30 gpurun_out/${T}_gpu_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.txt 2>&1 || { tail -10 gpurun_out/${T}_smoke.txt; exit 1; }
tail -1 gpurun_out/${T}_smoke.txt
timeout -k 10 600 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print('value', d['value'], d['ms_per_step'], 'packed', d['packed_obs']['value'], 'alt', d['alt_obs_dtype']['value'], 'cpu', d['cpu_baseline']['value'])" gpurun_out/${T}_bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/${T}_prof.log 2>&1 || { tail -5 gpurun_out/${T}_prof.log; exit 1; }
echo prof ok
timeout -k 10 300 python tools/bench_marl.py > gpurun_out/${T}_marl.json 2> gpurun_out/${T}_marl.err || { tail -5 gpurun_out/${T}_marl.err; exit 1; }
cat gpurun_out/${T}_marl.json

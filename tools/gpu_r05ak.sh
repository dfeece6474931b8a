#!/bin/bash
# Round 5: A2C acting as HIP graphs (act_graph): the marl GPU tests, then the loop with and without.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=r05ak
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_marl.py > gpurun_out/${T}_tests.txt 2>&1 \
  || { tail -30 gpurun_out/${T}_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_tests.txt
for r in 1 2; do
  timeout -k 10 300 python tools/bench_marl.py > gpurun_out/${T}_marl_eager.json 2> gpurun_out/${T}_marl.err || { tail -5 gpurun_out/${T}_marl.err; exit 1; }
  timeout -k 10 300 python tools/bench_marl.py --act-graph > gpurun_out/${T}_marl_actgraph.json 2> gpurun_out/${T}_marl.err || { tail -5 gpurun_out/${T}_marl.err; exit 1; }
  python -c "
import json
for n in ('eager','actgraph'):
    d=json.load(open('gpurun_out/${T}_marl_'+n+'.json')); print(n, d['env_steps_per_s'], d['ms_per_update'])"
done

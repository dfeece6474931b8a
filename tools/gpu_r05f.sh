#!/bin/bash
# Round 5: A2C learner update as a HIP graph (GPU tests of tests/test_marl.py, then bench_marl graph vs eager), and
# the render's layer-loop unroll variants (A/B against the in-tree library).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_marl.py > gpurun_out/r05f_marl_tests.txt 2>&1 \
  || { tail -40 gpurun_out/r05f_marl_tests.txt; exit 1; }
tail -2 gpurun_out/r05f_marl_tests.txt
timeout -k 10 300 python tools/bench_marl.py > gpurun_out/r05f_marl_graph.json 2> gpurun_out/r05f_marl_graph.err || { tail -20 gpurun_out/r05f_marl_graph.err; exit 1; }
cat gpurun_out/r05f_marl_graph.json
timeout -k 10 300 python tools/bench_marl.py --eager > gpurun_out/r05f_marl_eager.json 2> gpurun_out/r05f_marl_eager.err || { tail -20 gpurun_out/r05f_marl_eager.err; exit 1; }
cat gpurun_out/r05f_marl_eager.json
bash tools/ab_run.sh LU2 LU4 LU8 || exit 1

#!/bin/bash
# A2C learner with split-K weight gradients: GPU marl tests, throughput, profile.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_marl.py > gpurun_out/r04l_marl_tests.txt 2>&1 || { tail -20 gpurun_out/r04l_marl_tests.txt; exit 1; }
tail -2 gpurun_out/r04l_marl_tests.txt
timeout -k 10 300 python tools/bench_marl.py > gpurun_out/r04l_marl.json 2> gpurun_out/r04l_marl.err || { tail -5 gpurun_out/r04l_marl.err; exit 1; }
cat gpurun_out/r04l_marl.json
timeout -k 10 300 python tools/prof_a2c.py --updates 3 > gpurun_out/r04l_prof_a2c2.txt 2>&1 || exit 1
grep -v Warning gpurun_out/r04l_prof_a2c2.txt | head -32 | tail -28

#!/bin/bash
# Round 5: capacities raised (64 layers, 32 actions, 64 positions per agent; ABI 4): the GPU suite incl. the wide40
# reference fixtures and the batched wide40 parity.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=r05w
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > gpurun_out/${T}_gpu_tests.txt 2>&1 \
  || { tail -30 gpurun_out/${T}_gpu_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_gpu_tests.txt
timeout -k 10 300 python -u -m pytest -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k wide40 -v > gpurun_out/${T}_wide40.txt 2>&1 || { tail -30 gpurun_out/${T}_wide40.txt; exit 1; }
grep -E "PASS|FAIL" gpurun_out/${T}_wide40.txt

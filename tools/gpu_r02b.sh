#!/bin/bash
# round 2: plugin-surface parity first (new fixtures + batched oracle runs), then the whole GPU suite
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "eight_puzzle or narrow_corridor or obs_test or puzzle_dest_crash or corridor_quantity" > gpurun_out/tb1.log 2>&1
rc=$?; tail -25 gpurun_out/tb1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tb2.log 2>&1
rc=$?; tail -5 gpurun_out/tb2.log; exit $rc

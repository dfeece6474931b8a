#!/bin/bash
# Round 5: the full-batch final-state parity test (8,704 envs of the B = 65,536 timed mode against the C oracle).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 900 --timeout-method thread tests/test_gpu_timed_path.py -k final_state_of_every_env > gpurun_out/r05m_final_state.txt 2>&1 \
  || { tail -30 gpurun_out/r05m_final_state.txt; exit 1; }
tail -3 gpurun_out/r05m_final_state.txt

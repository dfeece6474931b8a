#!/bin/bash
# k_replay_done queue after each wave's first env: timed-path + parity subset, C3 A/B against the fixed stride.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_timed_path.py tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/t_r03n.log 2>&1 || { tail -30 gpurun_out/t_r03n.log; exit 1; }
tail -1 gpurun_out/t_r03n.log
./tools/ab_run.sh RPDQ0 || exit 1
echo done

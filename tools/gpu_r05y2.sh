#!/bin/bash
# Round 5: deferred replay flag (MFG_STEP_DEFER_REPLAY): its parity test, the A2C tests, then the A2C loop throughput.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=r05y2
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 200 --timeout-method thread tests/test_gpu_timed_path.py -k "deferred or fused_k8" tests/test_marl.py > gpurun_out/${T}_tests.txt 2>&1 \
  || { tail -30 gpurun_out/${T}_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_tests.txt
timeout -k 10 300 python tools/bench_marl.py > gpurun_out/${T}_marl.json 2> gpurun_out/${T}_marl.err || { tail -5 gpurun_out/${T}_marl.err; exit 1; }
cat gpurun_out/${T}_marl.json

#!/bin/bash
# In-tree library (learner kernels, k_logic split, MW store policy): GPU suite, smoke, every BASELINE config.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > gpurun_out/r04q_gpu_tests.txt 2>&1 \
  || { tail -30 gpurun_out/r04q_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/r04q_gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04q_smoke.txt 2>&1 || { tail -10 gpurun_out/r04q_smoke.txt; exit 1; }
tail -1 gpurun_out/r04q_smoke.txt
bash tools/bench_configs.sh r04q

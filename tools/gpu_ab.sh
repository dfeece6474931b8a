#!/bin/bash
# A/B timing of engine variants (tools/ab_run.sh) and, for the variant named by PARITY_LIB, the timed-path and
# fixture parity tests run on that library.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/ab_run.sh "$@" || exit 1
if [ -n "$PARITY_LIB" ]; then
  MFG_HIP_LIB=build/ablate/libmfg_hip_$PARITY_LIB.so timeout -k 10 400 python -u -m pytest tests/test_gpu_timed_path.py \
    tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_ab_$PARITY_LIB.log 2>&1 \
    || { tail -30 gpurun_out/t_ab_$PARITY_LIB.log; exit 1; }
  tail -1 gpurun_out/t_ab_$PARITY_LIB.log
fi

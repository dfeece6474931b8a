#!/bin/bash
# Dirt write-back skip (H_DIRT_TOUCH): parity on the dirt specs, C2/C4/C5 A/B against the REF library, C5 k_logic PMC.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=r06dw
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_timed_path.py > gpurun_out/${T}_tests.txt 2>&1 \
  || { tail -30 gpurun_out/${T}_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_tests.txt
AB_TAG=c4_ AB_ARGS="--config alltest16.yaml --batch 32768 --steps 200 --warmup 50" bash tools/ab_run.sh REF > gpurun_out/${T}_c4.txt 2>&1 || exit 1
cat gpurun_out/${T}_c4.txt
AB_TAG=c2_ AB_ARGS="--config rooms4.yaml --batch 4096 --steps 400 --warmup 100" bash tools/ab_run.sh REF > gpurun_out/${T}_c2.txt 2>&1 || exit 1
cat gpurun_out/${T}_c2.txt
bash tools/c5_logic_pmc.sh ${T}c5 > gpurun_out/${T}_c5.txt 2>&1 || exit 1
tail -40 gpurun_out/${T}_c5.txt

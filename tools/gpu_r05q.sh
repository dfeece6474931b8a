#!/bin/bash
# Round 5: packed tests on the final packed rule; C3 with resets (OV2) and resets + per-step replay (RE2) beside the render.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=r05q
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_marl.py -m gpu > gpurun_out/${T}_tests.txt 2>&1 \
  || { tail -30 gpurun_out/${T}_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_tests.txt
bash tools/ab_run.sh OV2 RE2

#!/bin/bash
# PMC passes (tools/pmc_run.sh) for the f64 headline (C3) and for C4 (alltest16, 32,768 envs).
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/pmc_run.sh r04k_c3 && bash tools/pmc_run.sh r04k_c4 --config alltest16.yaml --batch 32768 && echo ok

#!/bin/bash
# Round-5 evidence, part two: PMC passes of the headline workload, then the per-config lines (C2-C5, C4 serial).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r05z}
bash tools/pmc_run.sh ${T}_c3 || exit 1
bash tools/bench_configs.sh ${T} || exit 1

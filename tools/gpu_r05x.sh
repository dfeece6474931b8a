#!/bin/bash
# Round 5: 128-word replay chunks (W2: -DRP_W2=1) vs 64-word chunks (in-tree): fixed replay workload (state sha must
# match) and the bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/replay_ab.sh W2 || exit 1
bash tools/ab_run.sh W2 || exit 1

#!/bin/bash
# Round 5: k_replay Jacobi seed from the band's acceptance rate (SEED) vs 3l/4 (in-tree): fixed replay workload (state
# sha must match) and the bench.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/replay_ab.sh SEED || exit 1
bash tools/ab_run.sh SEED || exit 1

#!/bin/bash
# k_replay SALU cuts on the fixed workload (exact variants: their final state sha must equal the base's)
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/replay_ab.sh "$@"

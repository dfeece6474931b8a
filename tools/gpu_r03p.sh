#!/bin/bash
# HEAD verification (GPU suite, smoke, default bench) + k_replay phase ablations (timing-only builds).
cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/gpu_verify.sh || exit 1
bash tools/ab_run.sh "$@" || exit 1

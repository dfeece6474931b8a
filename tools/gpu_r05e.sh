#!/bin/bash
# Round 5: C3 render ablations, second set (suppression handling, per-agent table init).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/ab_run.sh ONORESUP ONOINIT ONOPLACE || exit 1

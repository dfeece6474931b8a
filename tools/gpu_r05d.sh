#!/bin/bash
# Round 5: where the C3 render's time goes now (timing-only ablations of the render unit, tools/build_obs_variant.sh),
# against the in-tree library, 2 alternating rounds.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/ab_run.sh ONORAY ONOPLACE ONOSTORE ONODEDUP || exit 1

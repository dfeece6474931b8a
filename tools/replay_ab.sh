#!/bin/bash
# tools/replay_bench.py for the in-tree library and each build/ablate/libmfg_hip_<VARIANT>.so, alternating, 2 rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for r in 1 2; do
  for v in base "$@"; do
    lib=""; [ "$v" != base ] && lib="build/ablate/libmfg_hip_$v.so"
    MFG_HIP_LIB=$lib timeout -k 10 200 python tools/replay_bench.py > gpurun_out/rb_${v}_$r.json 2> gpurun_out/rb_${v}_$r.err \
      || { tail -5 gpurun_out/rb_${v}_$r.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/rb_${v}_$r.json')); print('$v', d['k_replay_ms_mean'], d['k_replay_ms_min'], d['state_sha'])"
  done
done

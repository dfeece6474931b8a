#!/bin/bash
# Round 5: packed entries queued from the flattened pass (in-tree) vs per-layer ballots (PKOLD): packed parity tests,
# then the C3 / C4 bench side lines (f32 dense, packed entries, fused projection) alternating.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=r05p
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_marl.py -m gpu > gpurun_out/${T}_tests.txt 2>&1 \
  || { tail -30 gpurun_out/${T}_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_tests.txt
for r in 1 2; do
  for v in base PKOLD; do
    lib=""; [ "$v" != base ] && lib="build/ablate/libmfg_hip_$v.so"
    for c in c3 c4; do
      args="--steps 400 --warmup 100"
      [ $c = c4 ] && args="--config alltest16.yaml --batch 32768 --steps 100 --warmup 30"
      MFG_HIP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline $args > gpurun_out/${T}_${c}_$v.json 2> gpurun_out/${T}_${c}_$v.err || { tail -5 gpurun_out/${T}_${c}_$v.err; exit 1; }
      python -c "
import json; d=json.load(open('gpurun_out/${T}_${c}_$v.json')); p=d['packed_obs']; a=d['alt_obs_dtype']
print('$c $v', round(d['value']/1e6,2), 'f32', round(a['value']/1e6,2), 'packed', round(p['value']/1e6,2), 'fused', round(p['fused_proj']['value']/1e6,2), 'dense+gemm', round(p['dense_f32_plus_proj']['value']/1e6,2))"
    done
  done
done

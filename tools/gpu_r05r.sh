#!/bin/bash
# Round 5: k_logic stages only the live dirt slots of the step prefix (in-tree) vs the whole prefix (NOTRIM):
# the GPU suite, then C2 / C4 / C5 alternating.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=r05r
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > gpurun_out/${T}_gpu_tests.txt 2>&1 \
  || { tail -30 gpurun_out/${T}_gpu_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_gpu_tests.txt
for r in 1 2; do
  for v in base NOTRIM; do
    lib=""; [ "$v" != base ] && lib="build/ablate/libmfg_hip_$v.so"
    for c in c2 c4 c5; do
      case $c in
        c2) args="--config rooms4.yaml --batch 4096 --steps 400 --warmup 100";;
        c4) args="--config alltest16.yaml --batch 32768 --steps 100 --warmup 30";;
        c5) args="--config grid128_64.yaml --batch 131072 --fuse 1 --steps 4 --warmup 2";;
      esac
      MFG_HIP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --alt-steps 0 --packed-steps 0 $args > gpurun_out/${T}_${c}_$v.json 2> gpurun_out/${T}_${c}_$v.err || { tail -5 gpurun_out/${T}_${c}_$v.err; exit 1; }
      python -c "
import json; d=json.load(open('gpurun_out/${T}_${c}_$v.json'))
print('$c $v', round(d['value']/1e6,3), d['ms_per_step'], {k: v.get('mean_launch_ms', v.get('ms_per_step')) for k, v in d['roofline']['kernels'].items()})"
    done
  done
done

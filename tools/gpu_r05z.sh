#!/bin/bash
# Round 5: maintainer BFS in the HBM pool clears only the nodes it visited (was: all nf entries before every search):
# BFS parity tests (pool variant on maint_rooms, grid128_64 fixtures + batched), the C5 line, then the C5 PMC
# FETCH/WRITE passes for k_logic's traffic.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=r05z
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "bfs or grid128_64 or maint" > gpurun_out/${T}_tests.txt 2>&1 \
  || { tail -30 gpurun_out/${T}_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_tests.txt
timeout -k 10 300 python bench.py --no-cpu-baseline --alt-steps 0 --packed-steps 0 --config grid128_64.yaml --batch 131072 --fuse 1 --steps 6 --warmup 2 > gpurun_out/${T}_c5.json 2> gpurun_out/${T}_c5.err || { tail -5 gpurun_out/${T}_c5.err; exit 1; }
python -c "
import json; d=json.load(open('gpurun_out/${T}_c5.json'))
print('c5', d['value'], d['ms_per_step'], {k: v.get('mean_launch_ms', v.get('ms_per_step')) for k, v in d['roofline']['kernels'].items()})"
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-profile --alt-steps 0 --packed-steps 0 --config grid128_64.yaml --batch 131072 --fuse 1"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmc_${T}_c5_fetch -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc_${T}_c5_fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/pmc_${T}_c5_write -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc_${T}_c5_write.log 2>&1 || exit 1
echo pmc done
# C4 with the per-step replay beside the render (default) vs one replay per call (NORE)
for r in 1 2; do
  for v in base NORE; do
    lib=""; [ "$v" != base ] && lib="build/ablate/libmfg_hip_$v.so"
    MFG_HIP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --alt-steps 0 --packed-steps 0 --config alltest16.yaml --batch 32768 --steps 100 --warmup 30 > gpurun_out/${T}_c4_$v.json 2> gpurun_out/${T}_c4_$v.err || { tail -5 gpurun_out/${T}_c4_$v.err; exit 1; }
    python -c "
import json; d=json.load(open('gpurun_out/${T}_c4_$v.json'))
print('c4 $v', d['value'], d['ms_per_step'], {k: v.get('mean_launch_ms', v.get('ms_per_step')) for k, v in d['roofline']['kernels'].items()})"
  done
done

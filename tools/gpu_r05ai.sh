#!/bin/bash
# Round 5: rocprofv3 kernel statistics of the C4 and C5 lines (per instantiation).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05ai_c4_prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --alt-steps 0 --packed-steps 0 --config alltest16.yaml --batch 32768 --steps 200 --warmup 50 > gpurun_out/r05ai_c4_prof.log 2>&1 || { tail -5 gpurun_out/r05ai_c4_prof.log; exit 1; }
echo c4 ok
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r05ai_c5_prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --alt-steps 0 --packed-steps 0 --config grid128_64.yaml --batch 131072 --fuse 1 --steps 6 --warmup 2 > gpurun_out/r05ai_c5_prof.log 2>&1 || { tail -5 gpurun_out/r05ai_c5_prof.log; exit 1; }
echo c5 ok

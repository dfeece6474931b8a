#!/bin/bash
# PMC counter passes for the bench workload (run on the GPU box). Each pass is its own rocprofv3 run
# with --kernel-trace only (no sys/runtime trace), as the MI355X guide prescribes.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
ARGS="--steps 16 --warmup 8 --no-cpu-baseline $*"
set -e
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d gpurun_out/pmc_sq -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc_sq.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc_write.log 2>&1
echo done

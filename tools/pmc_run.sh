#!/bin/bash
# PMC counter passes for the bench workload (run on the GPU box via gpurun). Each pass is its own
# rocprofv3 run with --kernel-trace only (no sys/runtime trace), as the MI355X guide prescribes; the
# TCC counters need separate passes (FETCH_SIZE and WRITE_SIZE do not fit one pass).
# usage: tools/pmc_run.sh TAG [bench args...]   -> gpurun_out/pmc_TAG_{sq,fetch,write}/
TAG=${1:-x}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
ARGS="--steps 64 --warmup 16 --no-cpu-baseline --no-profile --alt-steps 0 --packed-steps 0 $*"
set -e
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d gpurun_out/pmc_${TAG}_sq -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc_${TAG}_sq.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmc_${TAG}_fetch -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc_${TAG}_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/pmc_${TAG}_write -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc_${TAG}_write.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS -d gpurun_out/pmc_${TAG}_lds -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc_${TAG}_lds.log 2>&1
echo pmc done

#!/bin/bash
# Extra SQ passes (issue/activity breakdown) for the bench workload. usage: tools/pmc_sq2.sh TAG
TAG=${1:-x}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
ARGS="--steps 32 --warmup 8 --no-cpu-baseline --no-profile"
set -e
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CU_CYCLES -d gpurun_out/pmc_${TAG}_a -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc_${TAG}_a.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INST_CYCLES_SALU SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_CYCLES -d gpurun_out/pmc_${TAG}_b -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc_${TAG}_b.log 2>&1
echo ok

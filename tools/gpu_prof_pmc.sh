#!/bin/bash
# rocprofv3 kernel-trace stats of the default bench command, then the PMC passes and their summary.
# usage: tools/gpu_prof_pmc.sh TAG
TAG=${1:-x}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1 || { tail -20 gpurun_out/prof_$TAG.log; exit 1; }
./tools/pmc_run.sh $TAG || exit 1
python tools/pmc_summarize.py $TAG large8_b65536_f8 8 gpurun_out/pmc_$TAG.json || exit 1
echo all done

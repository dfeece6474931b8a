#!/bin/bash
# GPU evidence, part 2: PMC passes (summarised into profiles/pmc_TAG.json, so the bench line's
# roofline.traffic reads this build's counters) and the rocprofv3 kernel-trace summary of the default
# bench command. usage: tools/gpu_profile.sh TAG
TAG=${1:-x}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
./tools/pmc_run.sh "$TAG" || exit 1
python tools/pmc_summarize.py "$TAG" large8_b65536_f8 8 "gpurun_out/pmc_$TAG.json" || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "gpurun_out/prof_$TAG" -o run --output-format csv -- python3 bench.py --no-cpu-baseline > "gpurun_out/prof_$TAG.log" 2>&1 || { tail -20 "gpurun_out/prof_$TAG.log"; exit 1; }
find "gpurun_out/prof_$TAG" -name '*kernel_stats.csv' -exec cat {} \;
tail -1 "gpurun_out/prof_$TAG.log"

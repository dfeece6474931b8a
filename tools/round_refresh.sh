#!/bin/bash
# Round-end evidence on the GPU box, in the order the bench line needs it: the PMC passes first
# (summarised into gpurun_out/pmc_TAG.json and copied into this box's profiles/, so the bench line's
# roofline.traffic reads this build's counters), then the GPU tests, smoke, the default bench line and a
# rocprofv3 kernel-trace summary of the same command. usage: tools/round_refresh.sh TAG
TAG=${1:-r01}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
./tools/pmc_run.sh "$TAG" || exit 1
python tools/pmc_summarize.py "$TAG" large8_b65536_f8 8 "gpurun_out/pmc_$TAG.json" || exit 1
cp "gpurun_out/pmc_$TAG.json" profiles/pmc_r01.json
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "gpurun_out/t_$TAG.log" 2>&1 || { tail -30 "gpurun_out/t_$TAG.log"; exit 1; }
tail -1 "gpurun_out/t_$TAG.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "gpurun_out/smoke_$TAG.log" 2>&1 || { tail -20 "gpurun_out/smoke_$TAG.log"; exit 1; }
tail -1 "gpurun_out/smoke_$TAG.log"
timeout -k 10 400 python bench.py > "gpurun_out/bench_$TAG.json" 2> "gpurun_out/bench_$TAG.err" || { tail -20 "gpurun_out/bench_$TAG.err"; exit 1; }
cat "gpurun_out/bench_$TAG.json"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "gpurun_out/prof_$TAG" -o run --output-format csv -- python3 bench.py --no-cpu-baseline > "gpurun_out/prof_$TAG.log" 2>&1 || { tail -20 "gpurun_out/prof_$TAG.log"; exit 1; }
find "gpurun_out/prof_$TAG" -name '*kernel_stats.csv' -exec cat {} \;

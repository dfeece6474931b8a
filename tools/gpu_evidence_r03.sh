#!/bin/bash
# Round-3 evidence: -m gpu suite, smoke, the default bench line (full protocol, CPU baseline), the rocprofv3
# kernel-trace summary of the same command, the PMC passes, and the per-config lines.
# usage: tools/gpu_evidence_r03.sh TAG   -> gpurun_out/{t,smoke,bench,prof,pmc,bc}_TAG*
TAG=${1:-r03}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > "gpurun_out/t_$TAG.log" 2>&1 || { tail -30 "gpurun_out/t_$TAG.log"; exit 1; }
tail -1 "gpurun_out/t_$TAG.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "gpurun_out/smoke_$TAG.log" 2>&1 || { tail -20 "gpurun_out/smoke_$TAG.log"; exit 1; }
tail -1 "gpurun_out/smoke_$TAG.log"
timeout -k 10 500 python bench.py > "gpurun_out/bench_$TAG.json" 2> "gpurun_out/bench_$TAG.err" || { tail -20 "gpurun_out/bench_$TAG.err"; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_$TAG.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value'])"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "gpurun_out/prof_$TAG" -o run --output-format csv -- python3 bench.py --no-cpu-baseline > "gpurun_out/prof_$TAG.log" 2>&1 || { tail -20 "gpurun_out/prof_$TAG.log"; exit 1; }
find "gpurun_out/prof_$TAG" -name '*kernel_stats.csv' -exec head -12 {} \;
./tools/pmc_run.sh "$TAG" || exit 1
python tools/pmc_summarize.py "$TAG" large8_b65536_f8 8 "gpurun_out/pmc_$TAG.json" || exit 1
./tools/bench_configs.sh "$TAG" || exit 1
echo evidence done

#!/bin/bash
# f3 checks on the GPU box: packed-obs parity + A2C loop tests, the MARL loop throughput, a short bench line
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_marl.py tests/test_spec_abi.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/f3_t.log 2>&1; rc=$?
tail -15 gpurun_out/f3_t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_marl.py > gpurun_out/f3_marl.json 2> gpurun_out/f3_marl.err || { tail -20 gpurun_out/f3_marl.err; exit 1; }
cat gpurun_out/f3_marl.json
timeout -k 10 300 python bench.py --steps 400 --warmup 600 --alt-steps 0 --no-cpu-baseline > gpurun_out/f3_bench.json 2> gpurun_out/f3_bench.err || { tail -20 gpurun_out/f3_bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/f3_bench.json'));print(d['value'], d['packed_obs'])"

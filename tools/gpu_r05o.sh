#!/bin/bash
# Round 5: the serial attribution variant (parity on C4's config) and C4 per-kernel times with and without overlap.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "serial or pair_spill" > gpurun_out/r05o_tests.txt 2>&1 \
  || { tail -30 gpurun_out/r05o_tests.txt; exit 1; }
tail -1 gpurun_out/r05o_tests.txt
run() {  # name, timeout, args...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to python bench.py --no-cpu-baseline "$@" > gpurun_out/r05o_$name.json 2> gpurun_out/r05o_$name.err || { tail -5 gpurun_out/r05o_$name.err; return 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], {k: v.get('mean_launch_ms', v.get('ms_per_step')) for k, v in d['roofline']['kernels'].items()})" gpurun_out/r05o_$name.json $name
}
run c4 300 --config alltest16.yaml --batch 32768 --steps 200 --warmup 50 --alt-steps 0 --packed-steps 0 &&
run c4_serial 300 --config alltest16.yaml --batch 32768 --steps 200 --warmup 50 --alt-steps 0 --packed-steps 0 --serial

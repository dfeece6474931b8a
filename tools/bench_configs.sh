#!/bin/bash
# Per-config throughput on one GPU (the BASELINE configs other than the headline): bench.py --config runs,
# each at its per-GPU shard of the BASELINE batch (C4 262,144 / 8, C5 1,048,576 / 8).
# usage (GPU box via gpurun): tools/bench_configs.sh TAG
TAG=${1:-x}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
run() {  # name, timeout, args...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to python bench.py --no-cpu-baseline "$@" > gpurun_out/bc_${TAG}_$name.json 2> gpurun_out/bc_${TAG}_$name.err || { tail -5 gpurun_out/bc_${TAG}_$name.err; return 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline'].get('pipeline',{}).get('frac'))" gpurun_out/bc_${TAG}_$name.json $name
}
run c3 300 --steps 400 --warmup 100 --alt-steps 0 --packed-steps 0 &&
run c2 200 --config rooms4.yaml --batch 4096 --steps 400 --warmup 100 --alt-steps 0 --packed-steps 0 &&
run c4 300 --config alltest16.yaml --batch 32768 --steps 200 --warmup 50 --alt-steps 0 --packed-steps 0 &&
run c4_serial 300 --config alltest16.yaml --batch 32768 --steps 200 --warmup 50 --alt-steps 0 --packed-steps 0 --serial &&
run c5 500 --config grid128_64.yaml --batch 131072 --fuse 1 --steps 10 --warmup 3 --alt-steps 0 --packed-steps 0

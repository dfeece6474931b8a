#!/bin/bash
# C5 (grid128_64, B = 131,072, one step per call) k_logic HBM traffic per launch: the C5 bench line, then separate
# rocprofv3 FETCH_SIZE and WRITE_SIZE passes (--kernel-trace only), summarised per launch by tools/pmc_per_launch.py.
# usage (GPU box via gpurun): tools/c5_logic_pmc.sh TAG
T=${1:-c5}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline --alt-steps 0 --packed-steps 0 --config grid128_64.yaml --batch 131072 \
  --fuse 1 --steps 6 --warmup 2 > gpurun_out/${T}_c5.json 2> gpurun_out/${T}_c5.err || { tail -5 gpurun_out/${T}_c5.err; exit 1; }
ARGS="--steps 4 --warmup 2 --no-cpu-baseline --no-profile --alt-steps 0 --packed-steps 0 --config grid128_64.yaml --batch 131072 --fuse 1"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/pmc_${T}_fetch -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc_${T}_fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/pmc_${T}_write -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/pmc_${T}_write.log 2>&1 || exit 1
python tools/pmc_per_launch.py gpurun_out/pmc_${T}_fetch gpurun_out/pmc_${T}_write k_logic > gpurun_out/${T}_logic_traffic.json && cat gpurun_out/${T}_logic_traffic.json

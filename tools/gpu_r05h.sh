#!/bin/bash
# Round 5: C5 two-wave replay, ring size A/B (register-MT producer): in-tree (7 chunks per half, 5 envs per CU) vs 10
# and 16 chunks per half (4 envs per CU).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in base R16 R10; do
  lib=""; [ "$v" != base ] && lib="build/ablate/libmfg_hip_$v.so"
  MFG_HIP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --config grid128_64.yaml --batch 131072 --fuse 1 --steps 6 --warmup 3 --alt-steps 0 --packed-steps 0 > gpurun_out/r05h_c5_$v.json 2> gpurun_out/r05h_c5_$v.err || { tail -5 gpurun_out/r05h_c5_$v.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['kernels']['k_replay']['mean_launch_ms'])" gpurun_out/r05h_c5_$v.json $v
done

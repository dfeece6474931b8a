#!/bin/bash
# Round 5: A2C learner phases (device time per phase), and the C4 render in isolation (resets not overlapped:
# -DMFG_RESET_OVERLAP=0) beside the in-tree overlapped figure.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python tools/prof_a2c_phases.py > gpurun_out/r05i_a2c_phases.json 2> gpurun_out/r05i_a2c_phases.err || { tail -10 gpurun_out/r05i_a2c_phases.err; exit 1; }
cat gpurun_out/r05i_a2c_phases.json
for v in base OVL0; do
  lib=""; [ "$v" != base ] && lib="build/ablate/libmfg_hip_$v.so"
  MFG_HIP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --config alltest16.yaml --batch 32768 --steps 200 --warmup 50 --alt-steps 0 --packed-steps 0 > gpurun_out/r05i_c4_$v.json 2> gpurun_out/r05i_c4_$v.err || { tail -5 gpurun_out/r05i_c4_$v.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], {k: v.get('mean_launch_ms') for k, v in d['roofline']['kernels'].items() if isinstance(v, dict)})" gpurun_out/r05i_c4_$v.json $v
done

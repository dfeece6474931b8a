#!/bin/bash
# Round 5: flattened dense-obs stores (MFG_OBS_FLAT): the whole GPU suite (every dense render is exact), then A/B
# against the per-layer stores (NOFLAT) at C3 and C4, and the A2C phase profile.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=r05k
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > gpurun_out/${T}_gpu_tests.txt 2>&1 \
  || { tail -30 gpurun_out/${T}_gpu_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_gpu_tests.txt
bash tools/ab_run.sh NOFLAT || exit 1
for v in base NOFLAT; do
  lib=""; [ "$v" != base ] && lib="build/ablate/libmfg_hip_$v.so"
  MFG_HIP_LIB=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --config alltest16.yaml --batch 32768 --steps 200 --warmup 50 --alt-steps 0 --packed-steps 0 > gpurun_out/${T}_c4_$v.json 2> gpurun_out/${T}_c4_$v.err || { tail -5 gpurun_out/${T}_c4_$v.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], {k: v.get('mean_launch_ms') for k, v in d['roofline']['kernels'].items() if isinstance(v, dict)})" gpurun_out/${T}_c4_$v.json $v
done
timeout -k 10 300 python tools/prof_a2c_phases.py > gpurun_out/${T}_a2c_phases.json 2> gpurun_out/${T}_a2c_phases.err || { tail -10 gpurun_out/${T}_a2c_phases.err; exit 1; }
cat gpurun_out/${T}_a2c_phases.json

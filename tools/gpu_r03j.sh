#!/bin/bash
# A/B of the replay beside the last render (C3, C4), then the round-3 evidence (suite, smoke, bench, rocprof, PMC,
# configs).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_timed_path.py -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/t_r03j.log 2>&1 || { tail -30 gpurun_out/t_r03j.log; exit 1; }
tail -1 gpurun_out/t_r03j.log
./tools/ab_run.sh RSIDE0 || exit 1
for v in base RSIDE0; do
  lib=""; [ "$v" != base ] && lib="build/ablate/libmfg_hip_$v.so"
  MFG_HIP_LIB=$lib timeout -k 10 200 python bench.py --config alltest16.yaml --batch 32768 --steps 200 --warmup 50 --alt-steps 0 --packed-steps 0 --no-cpu-baseline > gpurun_out/c4_$v.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/c4_$v.json')); print('C4 $v', d['value'], d['ms_per_step'])"
done
./tools/gpu_evidence_r03.sh r03b

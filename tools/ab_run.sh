#!/bin/bash
# A/B timing of engine variants: tools/ab_run.sh VARIANT... (build/ablate/libmfg_hip_VARIANT.so, built by
# tools/build_variant.sh or tools/build_ablation.sh) against the in-tree library, alternating, 2 rounds each.
# AB_ARGS replaces the workload arguments (default: the headline C3 run, 800 timed steps); AB_TAG names the outputs.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for r in 1 2; do
  for v in base "$@"; do
    lib=""; [ "$v" != base ] && lib="build/ablate/libmfg_hip_$v.so"
    MFG_HIP_LIB=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --alt-steps 0 --packed-steps 0 \
      ${AB_ARGS:---steps 800 --warmup 200} > gpurun_out/ab_${AB_TAG}$v.json 2>/dev/null || exit 1
    python -c "
import json; d=json.load(open('gpurun_out/ab_${AB_TAG}$v.json'))
print('$v', round(d['value']/1e6,2), {k: v.get('mean_launch_ms', v.get('ms_per_step')) for k, v in d['roofline']['kernels'].items()})"
  done
done

#!/bin/bash
# Round 5: the long-ray render (grid128 full observability) parity tests first, then the whole GPU suite and the
# default bench line.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r05c}
timeout -k 10 600 python -u -m pytest -x -v -m gpu --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "grid128_full or long_ray" > gpurun_out/${T}_lr_tests.txt 2>&1 \
  || { tail -40 gpurun_out/${T}_lr_tests.txt; exit 1; }
tail -3 gpurun_out/${T}_lr_tests.txt
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > gpurun_out/${T}_gpu_tests.txt 2>&1 \
  || { tail -30 gpurun_out/${T}_gpu_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_gpu_tests.txt
timeout -k 10 600 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('value', d['value'], d['ms_per_step'], 'peak', r['peak_measured'], 'k', {k: v['mean_launch_ms'] for k, v in r['kernels'].items() if isinstance(v, dict) and 'mean_launch_ms' in v})" gpurun_out/${T}_bench.json
bash tools/ab_run.sh NORED || exit 1

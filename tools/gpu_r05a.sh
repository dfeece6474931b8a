#!/bin/bash
# Round 5, first GPU call: the launcher / RCCL tests (world 1 under torch.distributed.run), the k_replay occupancy
# curve on the fixed replay workload (the in-tree library = 8 waves per SIMD; W7/W6/W4 = the same kernel with its LDS
# slice padded to 7/6/4 waves), and the default bench line.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r05a}
timeout -k 10 900 python -u -m pytest -x -v -m gpu --timeout 600 --timeout-method thread tests/test_gpu_ranks.py > gpurun_out/${T}_ranks.txt 2>&1 \
  || { tail -40 gpurun_out/${T}_ranks.txt; exit 1; }
tail -3 gpurun_out/${T}_ranks.txt
bash tools/replay_ab.sh W7 W6 W4 || exit 1
timeout -k 10 600 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -20 gpurun_out/${T}_bench.err; exit 1; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print('value', d['value'], d['ms_per_step'], 'peak', r['peak_measured'], r['peak_measured_how'])" gpurun_out/${T}_bench.json

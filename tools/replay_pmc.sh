#!/bin/bash
# Instruction counts of k_replay on the fixed replay workload (tools/replay_bench.py): one rocprofv3 SQ pass
# (--kernel-trace only) per library, base (in-tree) and each build/ablate/libmfg_hip_<VARIANT>.so.
# usage (GPU box via gpurun): tools/replay_pmc.sh TAG VARIANT...
T=${1:-rp}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in base "$@"; do
  lib=""; [ "$v" != base ] && lib="build/ablate/libmfg_hip_$v.so"
  MFG_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
    -d gpurun_out/pmc_${T}_$v -o run --output-format csv -- python3 tools/replay_bench.py --reps 2 > gpurun_out/pmc_${T}_$v.log 2>&1 || exit 1
done
python - "$T" base "$@" <<'PY'
import csv, json, sys
from collections import defaultdict
from pathlib import Path
t, vs = sys.argv[1], sys.argv[2:]
out = {}
for v in vs:
    f = next(Path(f'gpurun_out/pmc_{t}_{v}').rglob('*counter_collection.csv'))
    acc = defaultdict(list)
    for row in csv.DictReader(open(f)):
        if row['Kernel_Name'].replace('void ', '').startswith('k_replay('):
            acc[row['Counter_Name']].append(float(row['Counter_Value']))
    out[v] = {k: sum(x) / len(x) for k, x in acc.items()}
print(json.dumps(out, indent=1))
PY

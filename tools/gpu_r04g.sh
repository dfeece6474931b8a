#!/bin/bash
# PMC of k_replay on the fixed workload for the in-tree library and variants: instruction mix and issue activity.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in base "$@"; do
  lib=""; [ "$v" != base ] && lib="$GRAFT_REPO_ROOT/build/ablate/libmfg_hip_$v.so"
  MFG_HIP_LIB=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_LDS \
    SQ_WAVE_CYCLES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY -d gpurun_out/r04g_pmc1_$v -o run --output-format csv \
    -- python3 tools/replay_bench.py --reps 2 > gpurun_out/r04g_pmc1_$v.log 2>&1 || { tail -5 gpurun_out/r04g_pmc1_$v.log; exit 1; }
  MFG_HIP_LIB=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC \
    SQ_WAIT_ANY SQ_INST_CYCLES_SALU SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -d gpurun_out/r04g_pmc2_$v -o run \
    --output-format csv -- python3 tools/replay_bench.py --reps 2 > gpurun_out/r04g_pmc2_$v.log 2>&1 || { tail -5 gpurun_out/r04g_pmc2_$v.log; exit 1; }
done
python - "$@" <<'PY'
import csv, glob, collections, sys
for v in ['base'] + sys.argv[1:]:
    out = {}
    for p in ('pmc1', 'pmc2'):
        f = glob.glob(f'gpurun_out/r04g_{p}_{v}/**/*counter_collection.csv', recursive=True)[0]
        agg = collections.defaultdict(list)
        for row in csv.DictReader(open(f)):
            if row['Kernel_Name'].startswith('k_replay(') or row['Kernel_Name'].split('(')[0].endswith('k_replay'):
                agg[row['Counter_Name']].append(float(row['Counter_Value']))
        out.update({c: round(sum(x) / len(x)) for c, x in agg.items()})
    print(v, out)
PY

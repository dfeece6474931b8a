#!/bin/bash
# Round-4: SALU/VALU issue-rate probe, the PMC counter list, and instruction counts of k_replay on the fixed workload
# (base and the draws-only ablation).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 120 build/issue_probe > gpurun_out/r04e_issue_probe.txt 2>&1 || { cat gpurun_out/r04e_issue_probe.txt; exit 1; }
cat gpurun_out/r04e_issue_probe.txt
timeout -s KILL 60 rocprofv3 -L > gpurun_out/r04e_counters.txt 2>&1 || true
grep -o "SQ_[A-Z_0-9]*" gpurun_out/r04e_counters.txt | sort -u | tr '\n' ' ' | head -c 3000; echo
for v in base NOSWAPTW; do
  lib=""; [ "$v" != base ] && lib="$GRAFT_REPO_ROOT/build/ablate/libmfg_hip_$v.so"
  MFG_HIP_LIB=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
    SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY -d gpurun_out/r04e_pmc_$v -o run --output-format csv \
    -- python3 tools/replay_bench.py --reps 2 > gpurun_out/r04e_pmc_$v.log 2>&1 || { tail -5 gpurun_out/r04e_pmc_$v.log; exit 1; }
done
python - <<'PY'
import csv, glob, collections
for v in ('base', 'NOSWAPTW'):
    f = glob.glob(f'gpurun_out/r04e_pmc_{v}/**/*counter_collection.csv', recursive=True)[0]
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for row in csv.DictReader(open(f)):
        k = row['Kernel_Name'].split('(')[0]
        if 'k_replay' in k:
            agg[k][row['Counter_Name']].append(float(row['Counter_Value']))
    for k, d in agg.items():
        print(v, k, {c: round(sum(x) / len(x)) for c, x in d.items()})
PY

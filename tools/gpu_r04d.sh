#!/bin/bash
# Round-4 k_replay attribution on a fixed workload (tools/replay_bench.py: identical records, debt 69 per env) and
# the WRITE_SIZE / FETCH_SIZE calibration of k_logic's store widths (tools/wcal.hip).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/replay_ab.sh SINK0 NODEBT NOTWIST NOSWAP NOSWAPTW NOFWD NOFWDS NOFWDT NOJAC || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/wcal_w -o run --output-format csv -- build/wcal \
  > gpurun_out/wcal_w.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/wcal_f -o run --output-format csv -- build/wcal \
  > gpurun_out/wcal_f.log 2>&1 || exit 1
python - <<'PY'
import csv, glob, collections
for tag in ('w', 'f'):
    f = glob.glob(f'gpurun_out/wcal_{tag}/**/*counter_collection.csv', recursive=True)[0]
    agg = collections.defaultdict(list)
    for row in csv.DictReader(open(f)):
        agg[row['Kernel_Name'].split('(')[0]].append(float(row['Counter_Value']))
    for k, v in agg.items():
        print(tag, k, [round(x, 1) for x in v])
PY

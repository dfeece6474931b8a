#!/bin/bash
# A/B of the k_obs obs-store variants: GPU parity of the in-tree build, timing of the in-tree build
# against build/var variants (tools/build_variants.sh NT0:-DMFG_OBS_NT=0), and the WRITE_SIZE pass of the
# in-tree build. The packed-row variants in DESIGN.md were measured with this script on a kernel revision
# that had them (dropped). usage: tools/pack_probe.sh [VARIANT ...]   (default NT0)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_pack.log 2>&1 || { tail -30 gpurun_out/t_pack.log; exit 1; }
tail -1 gpurun_out/t_pack.log
./tools/variant_run.sh ${@:-NT0} > gpurun_out/pk_var.log 2>&1 || { cat gpurun_out/pk_var.log; exit 1; }
cat gpurun_out/pk_var.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/pmc_pk_write -o run --output-format csv -- python3 bench.py --steps 64 --warmup 16 --no-cpu-baseline --no-profile > gpurun_out/pmc_pk_write.log 2>&1 || { tail gpurun_out/pmc_pk_write.log; exit 1; }
python - <<'P'
import csv,glob,collections
f=glob.glob('gpurun_out/pmc_pk_write/**/*counter_collection.csv',recursive=True)[0]
d=collections.defaultdict(list)
for r in csv.DictReader(open(f)): d[r['Kernel_Name'].split('(')[0][:30]].append(float(r['Counter_Value']))
for k,v in d.items(): print(k, sum(v)/len(v)*1024)
P

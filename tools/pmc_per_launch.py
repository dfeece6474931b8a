#!/usr/bin/env python3
"""Per-launch HBM traffic of one kernel family from a FETCH_SIZE pass and a WRITE_SIZE pass (rocprofv3 csv dirs):
GB per launch in dispatch order, per template instance, HBM bytes = FETCH_SIZE x 2 + WRITE_SIZE (KiB; gfx950's
FETCH_SIZE counts half the bytes of wide coalesced reads, MI355X_MICROARCH.md "HBM").
usage: tools/pmc_per_launch.py FETCH_DIR WRITE_DIR KERNEL_PREFIX"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path


def load(d, counter, prefix):
    f = next(Path(d).rglob('*counter_collection.csv'))
    per = defaultdict(list)
    with open(f) as fh:
        for row in csv.DictReader(fh):
            name = row['Kernel_Name'].replace('void ', '')
            if not name.startswith(prefix) or row['Counter_Name'] != counter:
                continue
            per[name.split('(')[0]].append((int(row['Dispatch_Id']), float(row['Counter_Value'])))
    return {k: [v for _, v in sorted(x)] for k, x in per.items()}


def main():
    fd, wd, prefix = sys.argv[1:4]
    fe, wr = load(fd, 'FETCH_SIZE', prefix), load(wd, 'WRITE_SIZE', prefix)
    gb = lambda kib: round(kib * 1024 / 1e9, 3)
    out = {"what": f"{prefix} HBM traffic per launch (dispatch order), GB", "fetch_GB": {}, "write_GB": {},
           "hbm_GB": {}}
    for k in sorted(set(fe) | set(wr)):
        f, w = fe.get(k, []), wr.get(k, [])
        out["fetch_GB"][k] = [gb(x) for x in f]
        out["write_GB"][k] = [gb(x) for x in w]
        out["hbm_GB"][k] = [gb(2 * a + b) for a, b in zip(f, w)]
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()

#!/usr/bin/env python3
"""Summarise the rocprofv3 PMC passes of tools/pmc_run.sh into profiles/pmc_<tag>.json.

HBM bytes per launch = FETCH_SIZE x 2 (gfx950 reports half the bytes of wide coalesced reads,
MI355X_MICROARCH.md "HBM") + WRITE_SIZE; both counters are in KiB. bench.py reads
hbm_bytes_per_launch[<dominant kernel>] as roofline.traffic.
usage: tools/pmc_summarize.py TAG WORKLOAD FUSE [out.json]
"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def load(d):
    f = next(Path(d).rglob('*counter_collection.csv'))
    per = defaultdict(lambda: defaultdict(list))
    with open(f) as fh:
        for row in csv.DictReader(fh):
            name = row['Kernel_Name'].split('(')[0].replace('void ', '').split('<')[0].strip()
            per[name][row['Counter_Name']].append(float(row['Counter_Value']))
    return per


def main():
    tag, workload, fuse = sys.argv[1], sys.argv[2], int(sys.argv[3])
    out = Path(sys.argv[4]) if len(sys.argv) > 4 else ROOT / 'profiles' / f'pmc_{tag}.json'
    base = ROOT / 'gpurun_out'
    sq, fe, wr = load(base / f'pmc_{tag}_sq'), load(base / f'pmc_{tag}_fetch'), load(base / f'pmc_{tag}_write')
    lds = load(base / f'pmc_{tag}_lds') if (base / f'pmc_{tag}_lds').exists() else {}
    kernels, hbm = {}, {}
    for k in sorted(set(sq) | set(fe) | set(wr)):
        if not k.startswith('k_'):
            continue
        d = {}
        for src in (sq, fe, wr, lds):
            for c, vals in src.get(k, {}).items():
                d[c] = sum(vals) / len(vals)
        if 'FETCH_SIZE' in d and 'WRITE_SIZE' in d:
            d['hbm_bytes'] = 2 * d['FETCH_SIZE'] * 1024 + d['WRITE_SIZE'] * 1024
            hbm[k] = round(d['hbm_bytes'])
        if d.get('SQ_WAVE_CYCLES'):
            d['wait_any_frac'] = d['SQ_WAIT_ANY'] / d['SQ_WAVE_CYCLES']
            d['wait_inst_any_frac'] = d['SQ_WAIT_INST_ANY'] / d['SQ_WAVE_CYCLES']
        kernels[k] = {c: (round(v, 4) if isinstance(v, float) else v) for c, v in d.items()}
    res = {'workload': workload, 'fuse': fuse, 'tag': tag,
           'note': 'per-dispatch averages; FETCH_SIZE/WRITE_SIZE in KiB; hbm_bytes = 2*FETCH + WRITE',
           'hbm_bytes_per_launch': hbm, 'kernels': kernels}
    out.parent.mkdir(exist_ok=True)
    out.write_text(json.dumps(res, indent=1) + '\n')
    print(json.dumps(res['hbm_bytes_per_launch']))


if __name__ == '__main__':
    main()

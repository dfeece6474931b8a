#!/usr/bin/env python3
"""Register / occupancy table of every kernel in the engine library, from a gfx950 build with
-Rpass-analysis=kernel-resource-usage (what the compiler allocated: SGPRs, VGPRs, spills, waves per SIMD).
usage: python tools/kernel_resources.py [UNIT ...] > profiles/<tag>_kernel_resources.md
(default units: mfg_engine and mfg_obs_a, which holds the C2/C3 render instantiations)"""
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / 'marl-factory-grid_amd' / 'csrc'
FLAGS = ['--offload-arch=gfx950', '-O3', '-std=c++17', '-ffp-contract=off', '--cuda-device-only', '-c', '-o',
         '/dev/null', '-Rpass-analysis=kernel-resource-usage']
FIELDS = {'TotalSGPRs': 'sgpr', 'VGPRs': 'vgpr', 'SGPRs Spill': 'sgpr_spill', 'VGPRs Spill': 'vgpr_spill',
          'Occupancy [waves/SIMD]': 'waves', 'ScratchSize [bytes/lane]': 'scratch'}


def demangle(names):
    out = subprocess.run(['c++filt'], input='\n'.join(names), capture_output=True,
                         text=True).stdout.splitlines()
    return out if len(out) == len(names) else names


def unit_rows(unit):
    err = subprocess.run(['/opt/rocm/bin/hipcc', *FLAGS, str(CSRC / f'{unit}.hip')], capture_output=True,
                         text=True).stderr
    rows, cur = [], None
    for line in err.splitlines():
        m = re.search(r'remark: ([^:]+): (.*?) \[-Rpass-analysis', line)
        if not m:
            continue
        k, v = m.group(1).strip(), m.group(2).strip()
        if k == 'Function Name':
            cur = {'name': v}
            rows.append(cur)
        elif cur is not None and k in FIELDS:
            cur[FIELDS[k]] = v
    return rows


def main():
    units = sys.argv[1:] or ['mfg_engine', 'mfg_obs_a']
    print('| unit | kernel | SGPRs | VGPRs | SGPR spill | VGPR spill | scratch B/lane | waves/SIMD |')
    print('|---|---|---|---|---|---|---|---|')
    for u in units:
        rows = [r for r in unit_rows(u) if '_Z' in r['name'] and ('k_' in r['name'])]
        names = demangle([r['name'] for r in rows])
        for r, n in zip(rows, names):
            n = re.sub(r'\(.*', '', n.replace('(anonymous namespace)::', '')).replace('MfgDevSpec const*', '')
            print(f"| {u} | `{n}` | {r.get('sgpr')} | {r.get('vgpr')} | {r.get('sgpr_spill')} | {r.get('vgpr_spill')} "
                  f"| {r.get('scratch')} | {r.get('waves')} |")


if __name__ == '__main__':
    main()

#!/usr/bin/env python3
"""Writes the C5 level `grid128`: 128x128 with a '#' border, '#' on rows and
columns 32/64/96, and doors 'D' at (m,k) and (k,m) for m in {16,48,80,112}, k in {32,64,96}.
Result: 15153 non-wall cells of which 24 are doors. Floor cells use '-' like the reference's levels."""
from pathlib import Path

N = 128
g = [['-'] * N for _ in range(N)]
for i in range(N):
    for j in range(N):
        if i in (0, N - 1) or j in (0, N - 1) or i in (32, 64, 96) or j in (32, 64, 96):
            g[i][j] = '#'
for m in (16, 48, 80, 112):
    for k in (32, 64, 96):
        g[m][k] = 'D'
        g[k][m] = 'D'
out = Path(__file__).resolve().parent.parent / 'marl-factory-grid_amd' / 'mfg_amd' / 'levels' / 'grid128.txt'
out.write_text('\n'.join(''.join(r) for r in g))
nonwall = sum(c != '#' for r in g for c in r)
doors = sum(c == 'D' for r in g for c in r)
assert (nonwall, doors) == (15153, 24), (nonwall, doors)
print(out, nonwall, doors)

#!/usr/bin/env python3
"""Print the engine's per-config record layout and LDS slices (needs the GPU: mfg_create probes it)."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / 'marl-factory-grid_amd')]
from mfg_amd.spec import compile_spec  # noqa: E402
from mfg_amd.engine import Engine  # noqa: E402

for cfg in ['simple1.yaml', 'rooms4.yaml', 'large8.yaml', 'alltest16.yaml', 'default_large.yaml', 'maint_rooms.yaml',
            'grid128_64.yaml']:
    eng = Engine(compile_spec(cfg), 4)
    L = eng.layout
    print(cfg, {k: L[k] for k in ('size', 'o_mt', 'dirt_cap', 'lds_full', 'lds_logic', 'lds_obs', 'lds_replay',
                                  'bfs_off', 'bfs_bytes', 'max_pairs', 'scratch_bytes')})
    eng.close()

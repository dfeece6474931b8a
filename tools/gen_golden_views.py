#!/usr/bin/env python3
"""Golden fixtures for the host-side views of the facade: `Factory.summarize_state()`,
`Factory.summarize_header()` (factory.py:275-292, consumed by EnvRecorder, recorder.py:51,158) and the
render entity list `state.entities.render()` (factory.py:268, utils/utility_classes.py:23-35), recorded
from the REFERENCE (imported read-only from /root/reference through tools/standins/).

THIS SCRIPT RUNS ONLY IN THE DEVELOPMENT CONTAINER (it needs /root/reference). Outputs are small data
fixtures under tests/golden/views_<tag>.json.gz. Seeding as in tools/gen_golden.py.
"""
import argparse
import contextlib
import gzip
import io
import json
import random
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(REPO / 'tools' / 'standins'), '/root/reference']

from marl_factory_grid.environment.entity.object import Object  # noqa: E402
from marl_factory_grid.environment.factory import Factory  # noqa: E402

CFG_DIR = REPO / 'marl-factory-grid_amd' / 'mfg_amd' / 'configs'


def _plain(x):
    """JSON-safe copy (numpy scalars / tuples -> python)."""
    if isinstance(x, dict):
        return {str(k): _plain(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_plain(v) for v in x]
    if isinstance(x, (np.integer,)):
        return int(x)
    if isinstance(x, (np.floating,)):
        return float(x)
    if isinstance(x, np.bool_):
        return bool(x)
    return x


def render_list(env):
    out = []
    for r in env.state.entities.render():
        out.append(dict(name=str(r.name), pos=[int(r.pos[0]), int(r.pos[1])], value=float(r.value),
                        value_operation=str(r.value_operation), state=None if r.state is None else str(r.state),
                        id=int(r.id), real_name=str(r.real_name)))
    return out


def run(cfg_name, py_seed, n_steps, action_seed):
    random.seed(py_seed)
    Object._u_idx.clear()
    sink = io.StringIO()
    with contextlib.redirect_stdout(sink):
        env = Factory(str(CFG_DIR / cfg_name))
        env.reset()
    agents = env.state.entities._data['Agent']
    n_act = [len(a.actions) for a in agents]
    arng = np.random.default_rng(action_seed)
    rec = dict(config=cfg_name, py_seed=py_seed, action_seed=action_seed, steps=[])

    def record(actions, done):
        st, hd, rl = _plain(env.summarize_state()), _plain(env.summarize_header()), render_list(env)
        if rec['steps']:  # walls are static: kept once, in the first record ('static' placeholders after)
            first = rec['steps'][0]
            assert st['walls'] == first['state']['walls'] and hd['recWalls'] == first['header']['recWalls']
            nw = sum(1 for x in first['render'] if x['name'] == 'Wall')
            assert rl[:nw] == first['render'][:nw]
            st['walls'], hd['recWalls'], rl = 'static', 'static', ['static'] + rl[nw:]
        rec['steps'].append(dict(actions=actions, done=done, state=st, header=hd, render=rl))

    record(None, False)
    for _ in range(n_steps):
        acts = [int(arng.integers(0, n)) for n in n_act]
        with contextlib.redirect_stdout(sink):
            _, _, _, d, _ = env.step(acts)
        record(acts, bool(d))
        if d:
            with contextlib.redirect_stdout(sink):
                env.reset()
            record(None, False)
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--configs', default='simple1.yaml,rooms4.yaml,large8.yaml,alltest16.yaml,default_large.yaml')
    ap.add_argument('--seed', type=int, default=0)
    ap.add_argument('--steps', type=int, default=60)
    args = ap.parse_args()
    for cfg in args.configs.split(','):
        rec = run(cfg, args.seed, args.steps, 1000 + args.seed)
        out = REPO / 'tests' / 'golden' / f'views_{Path(cfg).stem}.json.gz'
        with gzip.open(out, 'wt') as f:
            json.dump(rec, f)
        print(out, len(rec['steps']), 'records')


if __name__ == '__main__':
    main()

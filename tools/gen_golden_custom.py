#!/usr/bin/env python3
"""Golden vectors for the custom-rule host fallback: runs the REFERENCE Factory on
mfg_amd/configs/custom_rules4.yaml with custom_modules_path = tests/custom_rules (the reference resolves
the custom classes with locate_and_import_class, utils/helpers.py:215-250) and records per step the
actions, rewards, done and info dict.

THIS SCRIPT RUNS ONLY IN THE DEVELOPMENT CONTAINER (it imports /root/reference read-only). Output:
tests/golden/custom_rules4_s{seed}.json.gz (data only).
"""
import contextlib
import gzip
import io
import json
import random
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent.parent
# the reference imports custom modules by path parts from its own package depth (/root/reference/x ->
# parts[3:]): /root/repo/tests/custom_rules/rules.py becomes `tests.custom_rules.rules` with /root/repo on
# sys.path
sys.path[:0] = [str(REPO / 'tools' / 'standins'), '/root/reference', str(REPO)]

from marl_factory_grid.environment.entity.object import Object  # noqa: E402
from marl_factory_grid.environment.factory import Factory  # noqa: E402
import marl_factory_grid.utils.config_parser as _cp  # noqa: E402

CFG = REPO / 'marl-factory-grid_amd' / 'mfg_amd' / 'configs' / 'custom_rules4.yaml'
CUSTOM = REPO / 'tests' / 'custom_rules'

# The reference's own loader cannot load a custom rule: _load_smth exits when BOTH built-in folders miss
# (`if (e1 and e2) or e3`, config_parser.py:238), even after the custom path found the class. The fixture
# records what the reference does once that lookup succeeds, in the reference's own search order: the
# built-in folders first (environment/, then modules/), the custom path last. A custom class that shadows a
# built-in name therefore resolves to the built-in, exactly as compile_spec / locate_custom_class do.
_orig_locate = _cp.locate_and_import_class


def _locate(name, folder=''):
    try:
        return _orig_locate(name, folder)
    except AttributeError:
        if Path(str(folder)).name != 'modules' or Path(str(folder)) == CUSTOM:
            raise
        # both built-in folders missed: answer with the custom path's class from the second built-in lookup,
        # so _load_smth sees e2 = None and keeps it instead of exiting
        return _orig_locate(name, CUSTOM)


_cp.locate_and_import_class = _locate


def run(py_seed, n_steps, action_seed):
    random.seed(py_seed)
    Object._u_idx.clear()
    sink = io.StringIO()
    with contextlib.redirect_stdout(sink):
        env = Factory(str(CFG), custom_modules_path=str(CUSTOM))
        env.reset()
    agents = env.state.entities._data['Agent']
    n_act = [len(a.actions) for a in agents]
    W = env.map.level_shape[1]
    arng = np.random.default_rng(action_seed)
    rec = dict(config=CFG.name, py_seed=py_seed, action_seed=action_seed, n_actions=n_act,
               rules=[r.name for r in env.state.rules], steps=[])
    episode, step = 0, 0
    for t in range(1, n_steps + 1):
        step += 1
        acts = [int(arng.integers(0, n)) for n in n_act]
        with contextlib.redirect_stdout(sink):
            _, _, r, d, info = env.step(acts)
        rec['steps'].append(dict(t=t, episode=episode, step=step, actions=acts, reward=[float(x) for x in r],
                                 done=bool(d), info={k: float(v) for k, v in info.items()},
                                 agent_pos=[[int(a.pos[0]), int(a.pos[1])] for a in agents]))
        if d:
            episode += 1
            step = 0
            with contextlib.redirect_stdout(sink):
                env.reset()
    return rec


def main():
    for seed in (0, 1):
        rec = run(seed, 450, 1000 + seed)
        dst = REPO / 'tests' / 'golden' / f'custom_rules4_s{seed}.json.gz'
        with gzip.open(dst, 'wt') as f:
            json.dump(rec, f)
        n_done = sum(s['done'] for s in rec['steps'])
        print('wrote', dst, 'episodes ended:', n_done, 'rules:', rec['rules'])


if __name__ == '__main__':
    main()

"""Test infrastructure: a `mfg_amd.views.Snapshot` of the C oracle's state (so the host-side views are
checked on CPU against the reference's own summarize_state / summarize_header / render fixtures, made by
tools/gen_golden_views.py), and the fixture comparison shared by the CPU and GPU view tests."""
import dataclasses
import gzip
import json

import golden_compare as G
from mfg_amd.views import Snapshot, render_entities, summarize_header, summarize_state

VIEW_FIXTURES = ['simple1', 'rooms4', 'large8', 'alltest16', 'default_large']


def load_views(tag):
    with gzip.open(G.GOLDEN / f'views_{tag}.json.gz', 'rt') as f:
        return json.load(f)


def oracle_snapshot(env):
    spec = env.spec
    pos, bat, st = env.agents()
    agents = []
    for a in range(spec.n_agents):
        ident, valid = int(st[a, 0]), bool(st[a, 1])
        name = 'Noop' if ident == -1 else 'Collisions' if ident == -2 else spec.action_classes[a][ident]
        agents.append((int(pos[a]), name, valid))
    opn, ttc = env.doors()
    ent, amt = env.entities()

    def grp(which, kind='plain'):
        out = []
        for h in env.group(which):
            cls, uid, cell, alive, reached = (int(x) for x in ent[h])
            if kind == 'dest':
                out.append((uid, cell, bool(reached)))
            elif kind == 'dirt':
                out.append((uid, cell, float(amt[h])))
            else:
                out.append((uid, cell))
        return out

    return Snapshot(step=int(env.header()[0]), agents=agents,
                    battery=[float(b) for b in bat] if spec.c.has_batteries else [],
                    doors=[(int(o), int(t)) for o, t in zip(opn, ttc)], items=grp(0), pods=grp(1), drops=grp(2),
                    dirt=grp(3, 'dirt'), dests=grp(4, 'dest'), machines=grp(5), maints=grp(6))


def render_dicts(spec, snap):
    out = []
    for r in render_entities(spec, snap):
        d = dataclasses.asdict(r)
        d.pop('aux')
        d['pos'] = [int(d['pos'][0]), int(d['pos'][1])]
        d['value'] = float(d['value'])
        out.append(d)
    return out


def expand(rec, first):
    """Re-insert the static walls a fixture keeps only in its first record."""
    if rec['state'].get('walls') != 'static':
        return rec
    nw = sum(1 for x in first['render'] if x['name'] == 'Wall')
    st = {k: (first['state']['walls'] if k == 'walls' else v) for k, v in rec['state'].items()}
    hd = {k: (first['header']['recWalls'] if k == 'recWalls' else v) for k, v in rec['header'].items()}
    return dict(rec, state=st, header=hd, render=first['render'][:nw] + rec['render'][1:])


def compare_record(spec, snap, rec, where):
    st = summarize_state(spec, snap)
    assert list(st) == list(rec['state']), f'{where}: summary keys {list(st)} != {list(rec["state"])}'
    for k in st:
        assert st[k] == rec['state'][k], f'{where}: summarize_state[{k}] differs'
    hd = summarize_header(spec, snap)
    assert hd == rec['header'], f'{where}: summarize_header differs'
    assert render_dicts(spec, snap) == rec['render'], f'{where}: render list differs'

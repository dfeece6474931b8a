"""Host-side views of one env's state: the reference's entity-group summaries and render list.

The engine keeps an env as one SoA record (csrc/mfg_device.h); the reference exposes it as entity
collections. This module rebuilds, from a neutral `Snapshot` of that record:

* `summarize_state` -- `Factory.summarize_state` (environment/factory.py:281-292): `{'step': n}` plus
  `<group name>.lower() -> [entity.summarize_state()]` for the groups in `Entities` order, then only the
  keys step/walls/doors/agents/items/dirtPiles/batteries survive (the lowercased 'dirtpiles' never
  matches 'dirtPiles', so dirt piles are always dropped, as in the reference);
* `summarize_header` -- `Factory.summarize_header` (:275-279): `rec_step` plus `rec<Name>` for Walls,
  DropOffLocations and ChargePods;
* `render_entities` -- `state.entities.render()` (:268; groups/global_entities.py:40-41): one
  `RenderEntity` (utils/utility_classes.py:23-35) per positioned entity, in group order;
* `GroupView` -- `Factory.__getitem__` (:131-132), a read-only snapshot of one collection.

Entity summaries follow entity/entity.py:201-209 (name, x, y, can_collide), agent.py:80-87 (valid,
action), doors/entitites.py:88-91 (state, time_to_close), batteries/entitites.py:71-74 and 116-119
(belongs_to, chargeLevel / charge_rate). Render entries follow wall.py:18, agent.py:120-139 (the 'move'
state is unreachable: action identifiers are class names), doors/entitites.py:93-95,
items/entitites.py:21-22 and 58-59, clean_up/entitites.py:45-46, batteries/entitites.py:113-114,
destinations/entitites.py:69-73, machines/entitites.py:78-79, maintenance/entities.py:138-139.
Groups come in `Entities` insertion order: Walls (level), Agents, then the YAML `Entities` order.
"""
from dataclasses import dataclass, field
from typing import List, Optional, Tuple

NO_POS = (-9999, -9999)  # c.VALUE_NO_POS
EW_ALIVE, EW_PRESENT, EW_REACHED, EW_NOPOS = 0x10000, 0x20000, 0x40000, 0xFFFF
SUMMARY_KEYS = ('step', 'walls', 'doors', 'agents', 'items', 'dirtPiles', 'batteries')  # factory.py:290


@dataclass
class Snapshot:
    """One env's state in engine-neutral form (cells are row-major x * W + y, -1 = no position)."""
    step: int
    agents: List[Tuple[int, str, bool]]              # (cell, state identifier, validity)
    battery: List[float]
    doors: List[Tuple[int, int]]                     # (open, time_to_close)
    items: List[Tuple[int, int]] = field(default_factory=list)       # (u_int, cell)
    pods: List[Tuple[int, int]] = field(default_factory=list)
    drops: List[Tuple[int, int]] = field(default_factory=list)
    dests: List[Tuple[int, int, bool]] = field(default_factory=list)  # (u_int, cell, reached)
    dirt: List[Tuple[int, int, float]] = field(default_factory=list)  # (u_int, cell, amount)
    machines: List[Tuple[int, int]] = field(default_factory=list)
    maints: List[Tuple[int, int]] = field(default_factory=list)


@dataclass
class RenderEntity:
    """utils/utility_classes.py:23-35 (aux, the agent's light map, is not rebuilt)."""
    name: str
    pos: Tuple[int, int]
    value: float = 1
    value_operation: str = 'none'
    state: Optional[str] = None
    id: int = 0
    aux: object = None
    real_name: str = 'none'


def agent_states(spec, actions, ev_act, ev_watch):
    """Per agent (identifier, validity) of `agent.state` after a step: the action result
    (states.py:187-196), overwritten by WatchCollisions (rules.py:303-307); an agent that did not act
    keeps the default Noop/valid state (entity.py:19)."""
    out = []
    for a in range(spec.n_agents):
        if int(ev_watch[a]) & 1:
            out.append(('Collisions', False))
        elif int(ev_act[a]) & 0x80:
            out.append((spec.action_classes[a][int(actions[a])], bool(int(ev_act[a]) & 1)))
        else:
            out.append(('Noop', True))
    return out


def snapshot_from_record(view, states):
    """Snapshot of an engine record (`engine.RecordView`); `states` from `agent_states` (or None after a
    reset: every agent Noop/valid)."""
    spec = view.spec
    A = spec.n_agents
    states = states or [('Noop', True)] * A
    pos = [int(x) for x in view.agent_pos()]
    opn, ttc, _ = view.doors()

    def grp(off_key, n_key, base_key, reached=False):
        n = view.hdr(n_key)
        if n <= 0:
            return []
        w = view.i32(view.L[off_key], n)
        base = view.hdr(base_key)
        out = []
        for k in range(n):
            x = int(w[k])
            if not x & EW_ALIVE:
                continue
            cell = -1 if (x & 0xFFFF) == EW_NOPOS else x & 0xFFFF
            out.append((base + k, cell, bool(x & EW_REACHED)) if reached else (base + k, cell))
        return out

    dpos, did, damt = view.dirt()
    dirt = [(int(i), -1 if (int(p) & 0xFFFF) == EW_NOPOS else int(p) & 0xFFFF, float(a))
            for p, i, a in zip(dpos, did, damt) if int(p) & EW_ALIVE]
    return Snapshot(
        step=view.hdr('step'), agents=[(pos[a], states[a][0], states[a][1]) for a in range(A)],
        battery=[float(x) for x in view.battery()] if spec.c.has_batteries else [],
        doors=[(int(o), int(t)) for o, t in zip(opn, ttc)],
        items=grp('o_items', 'n_items', 'item_base'), pods=grp('o_pods', 'n_pods', 'pod_base'),
        drops=grp('o_drops', 'n_drops', 'drop_base'), dests=grp('o_dests', 'n_dests', 'dest_base', True),
        dirt=dirt, machines=grp('o_machines', 'n_machines', 'machine_base'),
        maints=grp('o_maints', 'n_maints', 'maint_base'))


# ---- entity groups in Entities order --------------------------------------------------------------
def _xy(spec, cell):
    return NO_POS if cell < 0 else (cell // spec.W, cell % spec.W)


def _ent(name, spec, cell, can_collide, **extra):
    x, y = _xy(spec, cell)
    d = dict(name=name, x=int(x), y=int(y), can_collide=bool(can_collide))
    d.update(extra)
    return d


def group_order(spec):
    """`Entities` insertion order: Walls (level parse), Agents, then the YAML `Entities` groups."""
    return ['Walls', 'Agents'] + [g for g in spec.group_names if g not in ('Walls', 'Agents', 'Defaults')]


def group_summary(spec, snap, group):
    """`<Collection>.summarize_states()` (groups/objects.py:216-225) for one group, or None if the group
    has no per-entity summary here."""
    if group == 'Walls':
        return [_ent(f'Wall[{k}]', spec, int(c), True) for k, c in enumerate(spec.wall_cells)]
    if group == 'Agents':
        return [_ent(f'Agent[{n}]', spec, c, True, valid=bool(v), action=str(s))
                for n, (c, s, v) in zip(spec.agent_names, snap.agents)]
    if group == 'Batteries':
        return [dict(belongs_to=f'Agent[{n}]', chargeLevel=float(b)) for n, b in zip(spec.agent_names, snap.battery)]
    if group == 'Doors':
        return [_ent(f'Door[{k}]', spec, int(c), not o, state='open' if o else 'closed', time_to_close=int(t))
                for k, (c, (o, t)) in enumerate(zip(spec.door_cells, snap.doors))]
    if group == 'Items':
        return [_ent(f'Item[{i}]', spec, c, False) for i, c in snap.items]
    if group == 'ChargePods':
        return [_ent(f'ChargePod[{i}]', spec, c, False, charge_rate=float(spec.c.pod_charge_rate)) for i, c in snap.pods]
    if group == 'DropOffLocations':
        return [_ent(f'DropOffLocation[{i}]', spec, c, False) for i, c in snap.drops]
    if group == 'DirtPiles':
        return [_ent(f'DirtPile[{i}]', spec, c, False, amount=float(a)) for i, c, a in snap.dirt]
    if group == 'Destinations':
        return [_ent(f'Destination[{i}]', spec, c, False) for i, c, _ in snap.dests]
    if group == 'Machines':
        return [_ent(f'Machine[{i}]', spec, c, False) for i, c in snap.machines]
    if group == 'Maintainers':
        return [_ent(f'Maintainer[{i}]', spec, c, True) for i, c in snap.maints]
    return None


def summarize_state(spec, snap):
    out = {'step': int(snap.step)}
    for g in group_order(spec):
        s = group_summary(spec, snap, g)
        if s is not None:
            out[g.lower()] = s
    return {k: v for k, v in out.items() if k in SUMMARY_KEYS}


def summarize_header(spec, snap):
    header = {'rec_step': int(snap.step)}
    for g in group_order(spec):
        if g in ('Walls', 'DropOffLocations', 'ChargePods'):
            header[f'rec{g}'] = group_summary(spec, snap, g)
    return header


def render_entities(spec, snap):
    out = []
    for g in group_order(spec):
        if g == 'Walls':
            out += [RenderEntity('Wall', _xy(spec, int(c))) for c in spec.wall_cells]
        elif g == 'Agents':
            for i, (n, (c, s, v)) in enumerate(zip(spec.agent_names, snap.agents)):
                if s == 'Collisions':
                    name, st = 'agent_collision', None
                else:
                    name, st = 'Agent', ('idle' if s == 'Noop' else 'valid') if v else 'invalid'
                out.append(RenderEntity(name, _xy(spec, c), 1, 'none', st, i + 1, real_name=f'Agent[{n}]'))
        elif g == 'Doors':
            out += [RenderEntity('door_open' if o else 'door_closed', _xy(spec, int(c)), 1, 'none', 'blank', k + 1)
                    for k, (c, (o, _)) in enumerate(zip(spec.door_cells, snap.doors))]
        elif g == 'Items':
            out += [RenderEntity('Items', _xy(spec, c)) for _, c in snap.items if c >= 0]
        elif g == 'ChargePods':
            out += [RenderEntity('ChargePods', _xy(spec, c)) for _, c in snap.pods]
        elif g == 'DropOffLocations':
            out += [RenderEntity('DropOffLocations', _xy(spec, c)) for _, c in snap.drops]
        elif g == 'DirtPiles':
            out += [RenderEntity('DirtPiles', _xy(spec, c), min(0.15 + a, 1.5), 'scale') for _, c, a in snap.dirt]
        elif g == 'Destinations':
            out += [RenderEntity('Destinations', _xy(spec, c)) for _, c, r in snap.dests if not r]
        elif g == 'Machines':
            out += [RenderEntity('Machine', _xy(spec, c)) for _, c in snap.machines]
        elif g == 'Maintainers':
            out += [RenderEntity('Maintainer', _xy(spec, c)) for _, c in snap.maints]
    return out


class GroupView(list):
    """Read-only snapshot of one entity collection (`env['Doors']`, factory.py:131-132): a list of
    entity summaries with the collection's `name` and `summarize_states()`."""

    def __init__(self, name, entities):
        super().__init__(entities)
        self.name = name

    def summarize_states(self):
        return list(self)

    def __repr__(self):
        return f'{self.name}[{len(self)}]'


GROUP_ALIASES = {'Agent': 'Agents', 'Wall': 'Walls'}


def group_view(spec, snap, name):
    g = GROUP_ALIASES.get(name, name)
    if g not in group_order(spec):
        raise KeyError(name)
    s = group_summary(spec, snap, g)
    if s is None:
        raise KeyError(f'{name}: no per-entity view for this collection')
    return GroupView(g, s)


def render_ansi(spec, snap):
    """Text frame of the grid (the reference's pygame renderer is not part of this build): one character
    per cell, later groups drawn over earlier ones."""
    sym = {'Wall': '#', 'door_closed': 'D', 'door_open': 'd', 'Items': 'i', 'ChargePods': 'c',
           'DropOffLocations': 'o', 'DirtPiles': '.', 'Destinations': 'x', 'Machine': 'M', 'Maintainer': 'm',
           'Agent': 'A', 'agent_collision': '!'}
    grid = [[' '] * spec.W for _ in range(spec.H)]
    ents = render_entities(spec, snap)
    agents = [e for e in ents if e.name in ('Agent', 'agent_collision')]
    for e in [e for e in ents if e not in agents] + agents:
        x, y = e.pos
        if 0 <= x < spec.H and 0 <= y < spec.W:
            grid[x][y] = sym.get(e.name, '?')
    return '\n'.join(''.join(r) for r in grid)


RGB = {'Wall': (99, 110, 114), 'door_closed': (225, 112, 85), 'door_open': (250, 177, 160), 'Items': (253, 203, 110),
       'ChargePods': (0, 184, 148), 'DropOffLocations': (108, 92, 231), 'DirtPiles': (99, 72, 50),
       'Destinations': (232, 67, 147), 'Machine': (45, 52, 54), 'Maintainer': (214, 48, 49),
       'Agent': (9, 132, 227), 'agent_collision': (255, 0, 0)}


def render_rgb(spec, snap, bg=(223, 230, 233)):
    """(H, W, 3) uint8 frame: one pixel per cell, the render list drawn in order, agents last; dirt piles
    are scaled by their render value (clean_up/entitites.py:45-46)."""
    import numpy as np
    img = np.zeros((spec.H, spec.W, 3), np.uint8)
    img[:] = bg
    ents = render_entities(spec, snap)
    agents = [e for e in ents if e.name in ('Agent', 'agent_collision')]
    for e in [e for e in ents if e.name not in ('Agent', 'agent_collision')] + agents:
        x, y = e.pos
        if not (0 <= x < spec.H and 0 <= y < spec.W):
            continue
        col = np.asarray(RGB.get(e.name, (0, 0, 0)), np.float64)
        if e.value_operation == 'scale':
            col = np.asarray(bg, np.float64) + (col - np.asarray(bg, np.float64)) * min(float(e.value) / 1.5, 1.0)
        img[x, y] = col.astype(np.uint8)
    return img

"""Custom-plugin fallback: user Rule classes from `custom_modules_path` run on the host, on a
read-only view of the engine's state, and their Results are merged into the step's Result list.

Reference: `FactoryConfigParser._load_smth` / `locate_and_import_class` (utils/config_parser.py:213-250,
utils/helpers.py:215-250) resolve a YAML rule name in environment/, modules/ and then the custom path;
`StepRules` (utils/states.py:13-77) calls each rule's hooks in rule order; `summarize_step_results`
(environment/factory.py:222-259) folds the ordered Result list into rewards, info and done.

How it works here. The spec compiler keeps every built-in rule on the device and records a custom rule with
its position among them (`EnvSpec.host_rules`: slot = number of device rules before it). Per step the
`Factory` runs the device step, replays the device's Result list (`info.step_results`), calls the host
rules' `tick_pre_step` / `tick_step` / `tick_post_step` / `on_check_done` on a `StateView` of the record
after the step, inserts their Results at their rule position of each phase and folds the merged list
(`info.rebuild_rewards`, `info.fold_info`): rewards, info and done are then those of the reference.

Limits (what cannot run in or beside the kernel, rejected or documented):
  * custom rules are observers: the view is read-only (assigning to it raises), so a rule that moves
    entities, spawns or changes batteries is not supported;
  * a custom rule sees the state at the end of the device step. That equals the reference's view at its
    hook for everything the device rules do not change inside tick_step / tick_post_step (agent positions
    and states, items, dirt, destinations, batteries after their rule); door timers are updated by
    DoorAutoClose in tick_step. Where that differs -- a device rule later in the step than the custom rule's
    hook changes what it reads (`_MUTATORS`) -- the view refuses the read with `StaleStateError` instead of
    handing out the end-of-step value;
  * custom Entities and Actions are rejected (`UnsupportedSpec`): they would change the step itself.
"""
import dataclasses
import importlib.util
import sys
from pathlib import Path

from . import info as _info
from . import views as _views
from .spec import UnsupportedSpec

NO_POS = (-9999, -9999)

# Device rules that change state inside a step, by the hook phase they do it in (reference: doors/rules.py
# DoorAutoClose.tick_step, maintenance/rules.py MoveMaintainers.tick_step, batteries/rules.py
# BatteryDecharge.tick_step/tick_post_step, clean_up/rules.py RespawnDirt.tick_step and
# EntitiesSmearDirtOnMove.tick_post_step, destinations/rules.py DestinationReachReward.tick_step,
# items/rules.py RespawnItems.tick_step/tick_post_step, environment/rules.py WatchCollisions.tick_post_step).
# {rule: {phase: {group: attributes changed, or None for the whole group (membership, positions)}}}
_BATT = {'Batteries': ('charge_level', 'is_discharged')}
_MUTATORS = {
    'DoorAutoClose': {_info.TICK: {'Doors': ('is_open', 'is_closed', 'time_to_close')}},
    'MoveMaintainers': {_info.TICK: {'Maintainers': None}},
    'BatteryDecharge': {_info.TICK: _BATT, _info.POST: _BATT},
    'DoneAtBatteryDischarge': {_info.TICK: _BATT, _info.POST: _BATT},
    'RespawnDirt': {_info.TICK: {'DirtPiles': None}},
    'EntitiesSmearDirtOnMove': {_info.POST: {'DirtPiles': None}},
    'DestinationReachReward': {_info.TICK: {'Destinations': None}},
    'DoneAtDestinationReach': {_info.TICK: {'Destinations': None}},
    'RespawnItems': {_info.TICK: {'Items': None}, _info.POST: {'Items': None}},
    'WatchCollisions': {_info.POST: {'Agents': ('state',)}},
}


class StaleStateError(UnsupportedSpec):
    """A custom rule read state that a device rule later in the same step changes: the host view holds the
    end-of-step value, the reference would show the value at the custom rule's hook."""


def stale_state(spec, slot, phase):
    """{group: attrs | None} a host rule at rule position `slot` must not read in hook `phase`, and the device
    rule that makes each stale. The views are end-of-step snapshots (PRE: before the step), so everything a
    device rule changes at or after (phase, slot) is ahead of the reference's state at that hook. The TICK view
    carries the agents' action results as their states, so WatchCollisions' later states do not leak into it."""
    if phase in (_info.PRE, _info.DONE):
        return {}
    out = {}
    for i, name in enumerate(spec.rule_names):
        for ph, groups in _MUTATORS.get(name, {}).items():
            if ph < phase or (ph == phase and i < slot):
                continue
            for g, attrs in groups.items():
                if g == 'Agents' and ph != phase:
                    continue
                prev = out.get(g, ((), None))[0]
                merged = None if attrs is None or prev is None else tuple(prev) + tuple(attrs)
                out[g] = (merged, name)
    return out


def locate_custom_class(name, folder):
    """The class `name` from the .py files under `folder` (helpers.py:215-250 searches them with rglob and
    returns the first module that defines it). Modules are imported by file location."""
    folder = Path(folder).resolve()
    for path in sorted(folder.rglob('*.py')):
        if '__init__' in path.name:
            continue
        mod_name = 'mfg_custom_' + '_'.join(path.relative_to(folder).with_suffix('').parts)
        mod = sys.modules.get(mod_name)
        if mod is None:
            spec = importlib.util.spec_from_file_location(mod_name, path)
            mod = importlib.util.module_from_spec(spec)
            sys.modules[mod_name] = mod
            spec.loader.exec_module(mod)
        if hasattr(mod, name):
            return getattr(mod, name)
    return None


def level_map(spec):
    """The `lvl_map` handed to Rule.on_init (the reference passes its LevelParser, factory.py:127):
    `level_shape`, `pomdp_r` and the level text ('#' wall, 'D' door, '-' floor)."""
    sym = {0: '-', 1: '#', 2: 'D'}
    lv = spec.level.reshape(spec.H, spec.W)
    return _Frozen(level_shape=(spec.H, spec.W), pomdp_r=spec.pomdp_r,
                   level='\n'.join(''.join(sym[int(v)] for v in row) for row in lv))


class _Frozen:
    """Attribute bag that refuses assignment (host rules observe, they cannot change the device state)."""

    def __init__(self, _stale=None, **kw):
        object.__setattr__(self, '_d', kw)
        object.__setattr__(self, '_stale', _stale or {})

    def __getattr__(self, k):
        if k in self._stale:
            raise StaleStateError(self._stale[k])
        try:
            return self._d[k]
        except KeyError:
            raise AttributeError(f'{k!r} is not available on the host state view') from None

    def __setattr__(self, k, v):
        raise AttributeError('the host state view is read-only: custom rules cannot change the engine state')

    def __repr__(self):
        return self._d.get('name', type(self).__name__)


class EntityView(_Frozen):
    pass


class AgentView(EntityView):
    pass


class GroupView(list):
    """A collection (groups/collection.py): iterable entities, `name`, `by_pos`, `__getitem__` by index."""

    def __init__(self, name, ents):
        super().__init__(ents)
        self.name = name

    def by_pos(self, pos):
        return next((e for e in self if getattr(e, 'pos', None) == tuple(pos)), None)

    @property
    def positions(self):
        return [e.pos for e in self if hasattr(e, 'pos')]

    def __repr__(self):
        return f'{self.name}[{len(self)}]'


def _pos_dict(groups):
    """`entities.pos_dict` (groups/global_entities.py): entities by position, walls and agents first."""
    pos_dict = {}
    for g in ('Walls', 'Agents') + tuple(x for x in groups if x not in ('Walls', 'Agents', 'Batteries')):
        for e in groups[g]:
            if e.pos != NO_POS:
                pos_dict.setdefault(e.pos, []).append(e)
    return pos_dict


class StateView:
    """Read-only `Gamestate` stand-in for host rules: `curr_step`, `state[group]`, `state.entities.pos_dict`,
    `state.moving_entites` ... built from a `views.Snapshot` (one device->host record copy)."""

    def __init__(self, spec, snap):
        self.spec, self.snap = spec, snap
        self.curr_step = int(snap.step)
        W = spec.W

        def xy(cell):
            return NO_POS if cell < 0 else (int(cell) // W, int(cell) % W)

        agents = [AgentView(name=f'Agent[{n}]', pos=xy(c), x=xy(c)[0], y=xy(c)[1], identifier=f'Agent[{n}]',
                            state=_Frozen(identifier=s, validity=bool(v)), index=i)
                  for i, (n, (c, s, v)) in enumerate(zip(spec.agent_names, snap.agents))]
        groups = {'Walls': GroupView('Walls', [EntityView(name=f'Wall[{k}]', pos=xy(c), identifier=k)
                                               for k, c in enumerate(spec.wall_cells)]),
                  'Agents': GroupView('Agents', agents)}
        if 'Doors' in spec.group_names:
            groups['Doors'] = GroupView('Doors', [
                EntityView(name=f'Door[{k}]', pos=xy(c), identifier=k, is_open=bool(o), is_closed=not o,
                           time_to_close=int(t)) for k, (c, (o, t)) in enumerate(zip(spec.door_cells, snap.doors))])
        simple = {'Items': ('Item', snap.items), 'ChargePods': ('ChargePod', snap.pods),
                  'DropOffLocations': ('DropOffLocation', snap.drops), 'Machines': ('Machine', snap.machines),
                  'Maintainers': ('Maintainer', snap.maints)}
        for g, (cls, lst) in simple.items():
            if g in spec.group_names:
                groups[g] = GroupView(g, [EntityView(name=f'{cls}[{i}]', pos=xy(c), identifier=i) for i, c in lst])
        if 'DirtPiles' in spec.group_names:
            groups['DirtPiles'] = GroupView('DirtPiles', [EntityView(name=f'DirtPile[{i}]', pos=xy(c), identifier=i,
                                                                     amount=a) for i, c, a in snap.dirt])
        if 'Destinations' in spec.group_names:
            groups['Destinations'] = GroupView('Destinations', [
                EntityView(name=f'Destination[{i}]', pos=xy(c), identifier=i, reached=bool(r)) for i, c, r in snap.dests])
        if 'Batteries' in spec.group_names:
            groups['Batteries'] = GroupView('Batteries', [
                EntityView(name=f'Battery[{a.name}]', bound_entity=a, charge_level=float(b), is_discharged=b == 0)
                for a, b in zip(agents, snap.battery)])
        self._groups = groups
        self.entities = _Frozen(pos_dict=_pos_dict(groups), names=list(groups), floorlist_cells=len(spec.floor_cells))

    def restricted(self, stale, who):
        """This view with the reads in `stale` ({group: (attrs | None, device rule)}) refused for rule `who`."""
        if not stale:
            return self
        v = object.__new__(StateView)
        v.spec, v.snap, v.curr_step = self.spec, self.snap, self.curr_step
        v._whole = {}
        groups = dict(self._groups)
        for g, (attrs, dev) in stale.items():
            if g not in groups:
                continue
            msg = (f'custom rule {who!r} reads {g}{"" if attrs is None else "." + "/".join(attrs)}, which the '
                   f'device rule {dev!r} changes later in the step; the host view only holds the end-of-step state')
            if attrs is None:
                v._whole[g] = msg
            else:
                groups[g] = GroupView(g, [type(e)(_stale={a: msg for a in attrs}, **e._d) for e in groups[g]])
        v._groups = groups
        pos_msg = next((m for g, m in v._whole.items() if g != 'Batteries'), None)
        kw = dict(self.entities._d, pos_dict=_pos_dict(groups))
        v.entities = _Frozen(_stale={'pos_dict': pos_msg} if pos_msg else None, **kw)
        return v

    def __getitem__(self, key):
        key = {'Agent': 'Agents', 'Wall': 'Walls'}.get(key, key)
        if key in getattr(self, '_whole', {}):
            raise StaleStateError(self._whole[key])
        try:
            return self._groups[key]
        except KeyError:
            raise KeyError(f'{key}: no such collection in this env') from None

    def __contains__(self, key):
        return {'Agent': 'Agents', 'Wall': 'Walls'}.get(key, key) in self._groups

    @property
    def moving_entites(self):  # states.py:120-122 (sic)
        return list(self['Agents'])


def _as_res(r, phase, slot, names):
    """A user Result (utils/results.py shape: identifier, validity, reward, value, entity) -> info.Res."""
    ent = getattr(r, 'entity', None)
    ename = None if ent is None else getattr(ent, 'name', None)
    agent = names.index(ename) if ename in names else -1
    return _info.Res(ename, agent, str(r.identifier), reward=getattr(r, 'reward', None),
                     value=getattr(r, 'value', None), collision=bool(getattr(r, 'action_introduced_collision', False)),
                     valid=bool(getattr(r, 'validity', True)), phase=phase, slot=slot)


class HostRules:
    """The custom rules of one env, instantiated with their YAML kwargs (config_parser.py:246-248)."""

    def __init__(self, spec):
        self.spec = spec
        self.rules = [(slot, cls(**(kw or {}))) for slot, name, cls, kw in spec.host_rules]
        self.stale = [{ph: stale_state(spec, slot, ph) for ph in (_info.TICK, _info.POST)}
                      for slot, _, _, _ in spec.host_rules]
        self.rule_names = [name for _, name, _, _ in spec.host_rules]
        self.names = [f'Agent[{n}]' for n in spec.agent_names]

    def __bool__(self):
        return bool(self.rules)

    def on_init(self, view, lvl_map):
        for _, r in self.rules:
            r.on_init(view, lvl_map)

    def on_reset(self, view):
        for _, r in self.rules:
            r.on_reset(view)
            r.on_reset_post_spawn(view)

    def step_results(self, views):
        """Host results per phase, tagged with their rule slot (ahead of the device rule at that index).
        views: {phase: StateView} -- PRE: the state before the step (curr_step already advanced, agent states
        cleared, states.py:181-187); TICK: positions after the agents' actions with their action results as
        agent states; POST / DONE: the end of the step (WatchCollisions' states included)."""
        out = []
        for phase, hook in ((_info.PRE, 'tick_pre_step'), (_info.TICK, 'tick_step'), (_info.POST, 'tick_post_step'),
                            (_info.DONE, 'on_check_done')):
            for k, (slot, r) in enumerate(self.rules):
                view = views[phase].restricted(self.stale[k].get(phase), self.rule_names[k])
                for x in getattr(r, hook)(view) or []:
                    out.append(_as_res(x, phase, slot - 0.5, self.names))
        return out

    @staticmethod
    def merge(device, host):
        """One ordered Result list: by phase, then rule position (stable: in-rule order kept)."""
        return sorted(device + host, key=lambda r: (r.phase, r.slot))


def pre_snapshot(snap):
    """The state tick_pre_step sees (states.py:181-187): curr_step already advanced, agent states cleared."""
    return dataclasses.replace(snap, step=snap.step + 1, agents=[(c, 'Noop', True) for c, _, _ in snap.agents])


def fold_step(spec, host, actions, ev, pre, post, device_done):
    """One step with host rules: the device's Result list (from its event rows) merged with the host rules'
    Results, folded into (reward, done, info) like Factory.summarize_step_results (factory.py:222-259).
    pre: `pre_snapshot` of the state before the step; post: the state after it (agent states after
    WatchCollisions). tick_step sees `post` with the agents' action results as their states."""
    g = (lambda k: ev[k]) if isinstance(ev, dict) else (lambda k: getattr(ev, k))
    act = [int(x) for x in g('act')][:spec.n_agents]
    states = _views.agent_states(spec, actions, act, [0] * spec.n_agents)
    tick = dataclasses.replace(post, agents=[(c, s, v) for (c, _, _), (s, v) in zip(post.agents, states)])
    fv = StateView(spec, post)
    hres = host.step_results({_info.PRE: StateView(spec, pre), _info.TICK: StateView(spec, tick),
                              _info.POST: fv, _info.DONE: fv})
    merged = HostRules.merge(_info.step_results(spec, actions, ev), hres)
    reward = _info.rebuild_rewards(spec, merged)
    info = _info.rebuild_info(spec, actions, ev, reward, results=merged)
    done = bool(device_done) or any(r.valid for r in hres if r.phase == _info.DONE)
    return reward, done, info

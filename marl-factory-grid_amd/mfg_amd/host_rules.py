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
# BatteryDecharge.tick_step, clean_up/rules.py RespawnDirt.tick_step, destinations/rules.py
# DestinationReachReward.tick_step, environment/rules.py WatchCollisions.tick_post_step).
# {rule: {phase: {group: attributes changed, or None for the whole group (membership, positions)}}}
# Not listed, because they change nothing a view shows: RespawnItems (never spawns, SURVEY Q9: the item count
# stays at its limit, items/rules.py:28-43), EntitiesSmearDirtOnMove (never smears, Q1: move identifiers never
# match is_move, clean_up/rules.py:79), the tick_post_step of BatteryDecharge / DoneAtBatteryDischarge (it only
# paralyses agents, batteries/rules.py:66-87; charge changes in tick_step).
_BATT = {'Batteries': ('charge_level', 'is_discharged')}
_DOORS = {'Doors': ('is_open', 'is_closed', 'time_to_close')}
_REACHED = {'Destinations': ('reached', 'was_reached')}
_MUTATORS = {
    'DoorAutoClose': {_info.TICK: _DOORS},
    # maintainers open doors on their path through DoorUse inside their tick (maintenance/entities.py:91-100)
    'MoveMaintainers': {_info.TICK: {'Maintainers': None, **_DOORS}},
    'BatteryDecharge': {_info.TICK: _BATT},
    'DoneAtBatteryDischarge': {_info.TICK: _BATT},
    'RespawnDirt': {_info.TICK: {'DirtPiles': None}},
    'DestinationReachReward': {_info.TICK: _REACHED},
    'DoneAtDestinationReach': {_info.TICK: _REACHED},
    'WatchCollisions': {_info.POST: {'Agents': ('state',)}},
}
# DoneAtDestinationReach(condition='simultaneous') also unmarks reached destinations in on_check_done when not all
# are reached (destinations/rules.py:80-87), on any step, with or without a Result of its own
_DONE_SIMULTANEOUS = {_info.DONE: _REACHED}
_ON_RESULT = {'RespawnDirt', 'DestinationReachReward', 'DoneAtDestinationReach'}


class StaleStateError(UnsupportedSpec):
    """A custom rule read state that a device rule later in the same step changes: the host view holds the
    end-of-step value, the reference would show the value at the custom rule's hook. Raised from inside
    `Factory.step` after the device has executed the step: the Factory then refuses further steps until
    `reset()` (the step's rewards and info were never returned)."""


def stale_state(spec, slot, phase, fired=None):
    """{group: (attrs | None, device rule)} a host rule at rule position `slot` must not read in hook `phase`.
    The views are end-of-step snapshots (PRE: before the step), so everything a device rule changes at or after
    (phase, slot) is ahead of the reference's state at that hook. `fired`: the device rule indices that emitted a
    Result this step (None = assume every rule fired); a rule in `_ON_RESULT` that did not fire changed nothing.
    The TICK view carries the agents' action results as their states, so WatchCollisions' later states do not
    leak into it."""
    if phase == _info.PRE:
        return {}
    from . import abi
    out = {}
    for i, name in enumerate(spec.rule_names):
        muts = dict(_MUTATORS.get(name, {}))
        if name == 'DoneAtDestinationReach' and int(spec.c.rules[i].i[0]) == abi.DEST_SIMULTANEOUS:
            muts.update(_DONE_SIMULTANEOUS)  # not filtered by `fired`: the unmarking needs no Result
        elif name in _ON_RESULT and fired is not None and i not in fired:
            continue
        for ph, groups in muts.items():
            if ph < phase or (ph == phase and i < slot):
                continue
            if ph != _info.DONE and name in _ON_RESULT and fired is not None and i not in fired:
                continue
            for g, attrs in groups.items():
                if g == 'Agents' and ph != phase:
                    continue
                prev = out.get(g, ((), None))[0]
                merged = None if attrs is None or prev is None else tuple(prev) + tuple(attrs)
                out[g] = (merged, name)
    return out


def custom_modules(folder):
    """The modules of the .py files under `folder` (helpers.py:215-250 searches them with rglob), imported by file
    location, in path order. Module names carry a hash of the resolved folder, so two folders with a `rules.py`
    each never share a cached module; a module whose import raises is not left half-initialised in sys.modules."""
    import hashlib
    folder = Path(folder).resolve()
    tag = hashlib.sha1(str(folder).encode()).hexdigest()[:10]
    for path in sorted(folder.rglob('*.py')):
        if '__init__' in path.name:
            continue
        mod_name = f'mfg_custom_{tag}_' + '_'.join(path.relative_to(folder).with_suffix('').parts)
        mod = sys.modules.get(mod_name)
        if mod is None:
            spec = importlib.util.spec_from_file_location(mod_name, path)
            mod = importlib.util.module_from_spec(spec)
            sys.modules[mod_name] = mod
            try:
                spec.loader.exec_module(mod)
            except BaseException:
                sys.modules.pop(mod_name, None)
                raise
        yield mod


def locate_custom_class(name, folder):
    """The class `name` from the first module under `folder` that defines it (helpers.py:215-250)."""
    for mod in custom_modules(folder):
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


class PosDict(dict):
    """`entities.pos_dict` (groups/global_entities.py, a defaultdict(list)): entities by position, walls and
    agents first. `stale` {cell: message}: the cells whose entries a device rule later in the step changes
    (pre- and end-of-step positions of a whole-group mutator's entities); reading one raises StaleStateError,
    and so does walking the whole dict (its key set may differ from the hook's). Every other cell is exact."""

    def __init__(self, items=(), stale=None):
        super().__init__(items)
        self._stale = stale or {}

    def _check(self, pos):
        msg = self._stale.get(tuple(pos)) if isinstance(pos, (tuple, list)) else None
        if msg:
            raise StaleStateError(msg)

    def _check_all(self):
        if self._stale:
            raise StaleStateError(next(iter(self._stale.values())))

    def __missing__(self, pos):
        self._check(pos)
        return []

    def __getitem__(self, pos):
        self._check(pos)
        return super().__getitem__(pos)

    def get(self, pos, default=None):
        self._check(pos)
        return super().get(pos, default)

    def __contains__(self, pos):
        self._check(pos)
        return super().__contains__(pos)

    def __iter__(self):
        self._check_all()
        return super().__iter__()

    def keys(self):
        self._check_all()
        return super().keys()

    def values(self):
        self._check_all()
        return super().values()

    def items(self):
        self._check_all()
        return super().items()

    def __len__(self):
        self._check_all()
        return super().__len__()


def _pos_dict(groups, stale=None):
    """`entities.pos_dict` of the view's groups (see PosDict)."""
    pos_dict = {}
    for g in ('Walls', 'Agents') + tuple(x for x in groups if x not in ('Walls', 'Agents', 'Batteries')):
        for e in groups[g]:
            if e.pos != NO_POS:
                pos_dict.setdefault(e.pos, []).append(e)
    return PosDict(pos_dict, stale)


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
                EntityView(name=f'Destination[{i}]', pos=xy(c), identifier=i, reached=bool(r),
                           was_reached=(lambda r=bool(r): r)) for i, c, r in snap.dests])
        if 'Batteries' in spec.group_names:
            groups['Batteries'] = GroupView('Batteries', [
                EntityView(name=f'Battery[{a.name}]', bound_entity=a, charge_level=float(b), is_discharged=b == 0)
                for a, b in zip(agents, snap.battery)])
        self._groups = groups
        self.entities = _Frozen(pos_dict=_pos_dict(groups), names=list(groups), floorlist_cells=len(spec.floor_cells))

    def restricted(self, stale, who, before=None):
        """This view with the reads in `stale` ({group: (attrs | None, device rule)}) refused for rule `who`.
        A whole-group entry refuses the group and the pos_dict cells its entities occupy in this view or in
        `before` (the view before the step: where they stood at the hook); attribute entries refuse those
        attributes on the group's entities, and on the agents Batteries are bound to."""
        if not stale:
            return self
        v = object.__new__(StateView)
        v.spec, v.snap, v.curr_step = self.spec, self.snap, self.curr_step
        v._whole = {}
        groups = dict(self._groups)
        cells = {}
        for g, (attrs, dev) in stale.items():
            if g not in groups:
                continue
            msg = (f'custom rule {who!r} reads {g}{"" if attrs is None else "." + "/".join(attrs)}, which the '
                   f'device rule {dev!r} changes later in the step; the host view only holds the end-of-step state')
            if attrs is None:
                v._whole[g] = msg
                if g == 'DirtPiles' and before is not None and 'DirtPiles' in before._groups:
                    # RespawnDirt only adds piles or tops them up, at free cells (clean_up/groups.py:70-95,
                    # states.py:144-151); agents' Clean actions only lower amounts: the cells it changed are those
                    # with a new pile or a higher amount than before the step
                    was = {e.pos: e.amount for e in before._groups['DirtPiles']}
                    for e in groups[g]:
                        if e.pos != NO_POS and (e.pos not in was or e.amount > was[e.pos]):
                            cells.setdefault(e.pos, msg)
                elif g != 'Batteries':
                    for src in (groups[g], before._groups.get(g, ()) if before is not None else ()):
                        for e in src:
                            if e.pos != NO_POS:
                                cells.setdefault(e.pos, msg)
            else:
                groups[g] = GroupView(g, [type(e)(_stale={a: msg for a in attrs}, **e._d) for e in groups[g]])
        if 'Batteries' in groups and groups['Agents'] is not self._groups['Agents']:
            by_name = {a.name: a for a in groups['Agents']}  # bound_entity -> the restricted agent view
            groups['Batteries'] = GroupView('Batteries', [
                type(b)(_stale=b._stale, **dict(b._d, bound_entity=by_name.get(b._d['bound_entity'].name,
                                                                                 b._d['bound_entity'])))
                for b in groups['Batteries']])
        v._groups = groups
        kw = dict(self.entities._d, pos_dict=_pos_dict(groups, cells))
        v.entities = _Frozen(**kw)
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
        self._stale_cache = {}
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

    def step_results(self, views, fired=None):
        """Host results per phase, tagged with their rule slot (ahead of the device rule at that index).
        views: {phase: StateView} -- PRE: the state before the step (curr_step already advanced, agent states
        cleared, states.py:181-187); TICK: positions after the agents' actions with their action results as
        agent states; POST / DONE: the end of the step (WatchCollisions' states included).
        fired: device rule indices that emitted a Result this step (stale_state)."""
        out = []
        key = None if fired is None else frozenset(fired)
        for phase, hook in ((_info.PRE, 'tick_pre_step'), (_info.TICK, 'tick_step'), (_info.POST, 'tick_post_step'),
                            (_info.DONE, 'on_check_done')):
            for k, (slot, r) in enumerate(self.rules):
                cache = self._stale_cache.setdefault((k, phase), {})
                if key not in cache:
                    cache[key] = stale_state(self.spec, slot, phase, fired)
                view = views[phase].restricted(cache[key], self.rule_names[k], before=views[_info.PRE])
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
    dres = _info.step_results(spec, actions, ev)
    fired = {r.slot for r in dres if r.slot >= 0}
    hres = host.step_results({_info.PRE: StateView(spec, pre), _info.TICK: StateView(spec, tick),
                              _info.POST: fv, _info.DONE: fv}, fired)
    merged = HostRules.merge(dres, hres)
    reward = _info.rebuild_rewards(spec, merged)
    info = _info.rebuild_info(spec, actions, ev, reward, results=merged)
    done = bool(device_done) or any(r.valid for r in hres if r.phase == _info.DONE)
    return reward, done, info

"""Spec compiler: reference YAML config + level file -> `EnvSpec` (numpy tables + the C-ABI `MfgSpec`).

Mirrors the reference's config surface (same YAML schema, defaults and quirks):
  FactoryConfigParser       marl_factory_grid/utils/config_parser.py:16-274
  LevelParser.do_init       marl_factory_grid/utils/level_parser.py:62-102
  OBSBuilder layer naming   marl_factory_grid/utils/observation_builder.py:237-277
  RayCaster ray table       marl_factory_grid/utils/ray_caster.py:34-49,141-199
Classes are resolved by their reference name to an engine opcode; a class the engine does not implement
raises `UnsupportedSpec` (the reference would resolve custom classes reflectively, helpers.py:215-250).
"""
import ast
import ctypes as C
import math
from dataclasses import dataclass, field
from pathlib import Path
from typing import Dict, List, Optional

import numpy as np
import yaml

from . import abi

PKG_DIR = Path(__file__).resolve().parent
LEVELS_DIR = PKG_DIR / 'levels'
CONFIGS_DIR = PKG_DIR / 'configs'


class UnsupportedSpec(ValueError):
    pass


# ---- action catalogue: class name -> (opcode, arg, identifier, default valid, default fail) ----
# rewards: environment/rewards.py:1-5, modules/*/constants.py
_ACTIONS = {
    'Noop': (abi.ACT_NOOP, 0, 'Noop', -0.01, -0.01),
    'Charge': (abi.ACT_CHARGE, 0, 'do_charge_action', 0.1, -0.1),
    'Clean': (abi.ACT_CLEAN, 0, 'do_cleanup_action', 0.5, -0.1),
    'DestAction': (abi.ACT_DEST, 0, 'Destinations', 0.1, -0.1),
    'DoorUse': (abi.ACT_DOORUSE, 0, 'use_door', -0.0, -0.01),
    # ItemAction passes PICK_UP_FAIL as the valid reward and PICK_UP_VALID as the fail reward (Q8)
    'ItemAction': (abi.ACT_ITEM, 0, 'ITEMACTION', -0.1, 0.1),
    'MachineAction': (abi.ACT_MACHINE, 0, 'Maintain', 0.5, -0.1),
}
for _i, _n in enumerate(abi.DIR_NAMES):
    _ACTIONS[_n] = (abi.ACT_MOVE, _i, abi.DIR_IDENT[_i], -0.001, -0.05)
_MOVE_GROUPS = {'Move4': ['North', 'East', 'South', 'West'],
                'Move8': ['North', 'East', 'South', 'West', 'NorthEast', 'SouthEast', 'SouthWest', 'NorthWest']}
_NO_KWARGS = {'Charge', 'Clean', 'DestAction', 'MachineAction'}  # their __init__ takes no kwargs

# entity groups: YAML name -> (positional tag or None, spawn rule op or None)
_GROUPS = {
    'Batteries': (None, abi.RULE_SPAWN_BATTERIES),
    'ChargePods': (abi.TAG_PODS, abi.RULE_SPAWN_PODS),
    'Destinations': (abi.TAG_DESTS, abi.RULE_SPAWN_DESTS),
    'DirtPiles': (abi.TAG_DIRT, abi.RULE_SPAWN_DIRT),
    'Doors': (abi.TAG_DOORS, None),
    'DropOffLocations': (abi.TAG_DROPOFFS, abi.RULE_SPAWN_DROPOFFS),
    'GlobalPositions': (None, abi.RULE_SPAWN_GLOBALPOS),
    'Inventories': (None, abi.RULE_SPAWN_INVENTORIES),
    'Items': (abi.TAG_ITEMS, abi.RULE_SPAWN_ITEMS),
    'Machines': (abi.TAG_MACHINES, abi.RULE_SPAWN_MACHINES),
    'Maintainers': (abi.TAG_MAINTAINERS, abi.RULE_SPAWN_MAINTAINERS),
}
_POS_TAGS = {'Walls': abi.TAG_WALLS, **{k: v[0] for k, v in _GROUPS.items() if v[0] is not None}}

_RULES = {
    'DoorAutoClose': abi.RULE_DOOR_AUTOCLOSE, 'RespawnItems': abi.RULE_RESPAWN_ITEMS,
    'WatchCollisions': abi.RULE_WATCH_COLLISIONS, 'BatteryDecharge': abi.RULE_BATTERY_DECHARGE,
    'DoneAtBatteryDischarge': abi.RULE_DONE_BATTERY, 'DoneAtMaxStepsReached': abi.RULE_DONE_MAXSTEPS,
    'RespawnDirt': abi.RULE_RESPAWN_DIRT, 'EntitiesSmearDirtOnMove': abi.RULE_SMEAR_DIRT,
    'DoneOnAllDirtCleaned': abi.RULE_DONE_DIRT, 'DestinationReachReward': abi.RULE_DEST_REACH,
    'DoneAtDestinationReach': abi.RULE_DONE_DEST, 'MoveMaintainers': abi.RULE_MOVE_MAINTAINERS,
    'DoneAtMaintainerCollision': abi.RULE_DONE_MAINT_COLLISION, 'DoRandomInitialSteps': abi.RULE_RANDOM_INIT_STEPS,
}
# Destinations `spawnrule` classes (modules/destinations/rules.py:95-162)
_DEST_SPAWNRULES = {'SpawnDestinationOnAgent': abi.RULE_SPAWN_DEST_ON_AGENT,
                    'SpawnDestinationsPerAgent': abi.RULE_SPAWN_DEST_PER_AGENT}


def _literal_cells(values, H, W, what):
    """'(x, y)' strings (ast.literal_eval, config_parser.py:181 / destinations/rules.py:111) -> cell indices."""
    cells = []
    for v in values:
        xy = ast.literal_eval(v) if isinstance(v, str) else tuple(v)
        if len(xy) != 2 or not (0 <= int(xy[0]) < H and 0 <= int(xy[1]) < W):
            raise UnsupportedSpec(f'{what}: position {v!r} outside the {H}x{W} level')
        cells.append(int(xy[0]) * W + int(xy[1]))
    if len(cells) > abi.MAX_POSITIONS:
        raise UnsupportedSpec(f'{what}: more than {abi.MAX_POSITIONS} positions')
    return cells


def ray_table(d: int, n_rays: int = 100, degs: int = 360):
    """Ray offsets for a caster of radius d (= window diameter, Q13). Restates RayCaster.build_ray_targets
    (ray_caster.py:34-49, numpy round-half-even + unique rows) and bresenham_loop (ray_caster.py:141-199)."""
    north = np.array([0, -1]) * d
    thetas = [np.deg2rad(deg) for deg in np.linspace(-degs // 2, degs // 2, n_rays)[::-1]]
    rot = np.stack([[[math.cos(t), -math.sin(t)], [math.sin(t), math.cos(t)]] for t in thetas], 0)
    targets = np.unique(np.round(rot @ north), axis=0).astype(int)
    rays = []
    for tx, ty in targets:
        x1, y1, x2, y2 = 0, 0, int(tx), int(ty)
        steep = abs(y2 - y1) > abs(x2 - x1)
        if steep:
            x1, y1, x2, y2 = y1, x1, y2, x2
        swapped = x1 > x2
        if swapped:
            x1, x2, y1, y2 = x2, x1, y2, y1
        dx, dy = x2 - x1, y2 - y1
        err = int(dx / 2.0)
        ystep = 1 if y1 < y2 else -1
        y, pts = y1, []
        for x in range(x1, x2 + 1):
            pts.append((y, x) if steep else (x, y))
            err -= abs(dy)
            if err < 0:
                y += ystep
                err += dx
        if swapped:
            pts.reverse()
        rays.append(pts)
    return rays


def _n_abbr(n):
    return {1: 'st', 2: 'nd', 3: 'rd'}.get(n, 'th')


@dataclass
class EnvSpec:
    config_path: str
    level_name: str
    H: int
    W: int
    level: np.ndarray            # uint8 [H*W]: 0 floor, 1 wall, 2 door
    floor_cells: np.ndarray      # int32, row-major non-wall cells
    wall_cells: np.ndarray
    door_cells: np.ndarray
    pomdp_r: int
    ray_off: np.ndarray
    ray_pts: np.ndarray
    agent_names: List[str]       # 'Wolfgang', 'Wolfgang_the_0th', ...
    action_classes: List[List[str]]   # per agent, reference class names (info keys)
    action_idents: List[List[str]]    # per agent, Action.name (named_action_space)
    layer_names: List[List[str]]      # per agent, OBSBuilder.obs_layers
    rule_names: List[str]             # reference rule class names, spec order
    group_names: List[str]            # YAML entity group order
    individual_rewards: bool
    env_seed: int
    c: abi.MfgSpec = field(repr=False, default=None)
    _keep: list = field(repr=False, default_factory=list)

    @property
    def n_agents(self):
        return len(self.agent_names)

    @property
    def d(self):
        """window diameter (pomdp_r > 0); with pomdp_r == 0 the window is the level, see obs_hw"""
        return 2 * self.pomdp_r + 1

    @property
    def obs_hw(self):
        """(h, w) of one observation layer: (d, d), or the level shape with full observability
        (observation_builder.py:51)"""
        return (self.d, self.d) if self.pomdp_r else (self.H, self.W)

    @property
    def ray_radius(self):
        """RayCaster radius = min(obs_shape) (observation_builder.py:244; Q13)"""
        return min(self.obs_hw)

    @property
    def n_layers(self):
        return [len(x) for x in self.layer_names]

    @property
    def max_layers(self):
        return max(self.n_layers)

    @property
    def n_actions(self):
        return [len(x) for x in self.action_classes]


def _parse_level(path: Path):
    """helpers.py:168-183 parse_level + level_parser.py:46-60 argwhere order."""
    with open(path) as f:
        rows = [list(line.strip()) for line in f.readlines()]
    if len(set(len(r) for r in rows)) > 1:
        raise UnsupportedSpec('Every row of the level string must be of equal length.')
    arr = np.array(rows)
    H, W = arr.shape
    level = np.zeros((H, W), np.uint8)
    level[arr == '#'] = 1
    level[arr == 'D'] = 2
    walls = np.argwhere(arr == '#')
    doors = np.argwhere(arr == 'D')
    floor = np.argwhere(arr != '#')
    to_cells = lambda a: (a[:, 0] * W + a[:, 1]).astype(np.int32) if len(a) else np.zeros(0, np.int32)
    return H, W, level.reshape(-1), to_cells(floor), to_cells(walls), to_cells(doors)


def _parse_actions(conf_actions):
    """config_parser.py:133-177"""
    if isinstance(conf_actions, dict):
        kw = dict(conf_actions)
        names = list(conf_actions.keys())
    elif isinstance(conf_actions, list):
        kw = {}
        if any(isinstance(x, dict) for x in conf_actions):
            raise UnsupportedSpec('Actions list may not contain dicts (config_parser.py:153-154 raises)')
        names = list(conf_actions)
    else:
        raise UnsupportedSpec('Actions must be a list or a dict')
    expanded = []
    for a in names:
        if a == 'Defaults':
            expanded += ['Move8', 'Noop']
        else:
            expanded.append(a)
    classes, kwargs = [], {}
    for a in expanded:
        if a in _MOVE_GROUPS:
            for cls in _MOVE_GROUPS[a]:
                classes.append(cls)
                kwargs[cls] = kw.get(a) or {}
        elif a in _ACTIONS:
            classes.append(a)
        else:
            raise UnsupportedSpec(f'action class {a!r} is not implemented by the engine')
    out = []
    for cls in classes:
        k = kwargs.get(cls, kw.get(cls) or {}) or {}
        op, arg, ident, dv, df = _ACTIONS[cls]
        if k and cls in _NO_KWARGS:
            raise UnsupportedSpec(f'{cls} takes no kwargs (TypeError upstream)')
        unknown = set(k) - {'valid_reward', 'fail_reward', 'failed_dropoff_reward', 'valid_dropoff_reward'}
        if unknown:
            raise UnsupportedSpec(f'unknown kwargs for {cls}: {unknown}')
        vr = k.get('valid_reward')
        fr = k.get('fail_reward')
        act = dict(cls=cls, ident=ident, op=op, arg=arg,
                   valid=float(vr) if vr is not None else dv, fail=float(fr) if fr is not None else df,
                   aux0=0.1, aux1=-0.1)
        if cls == 'ItemAction':
            if k.get('valid_dropoff_reward') is not None:
                act['aux0'] = float(k['valid_dropoff_reward'])
            if k.get('failed_dropoff_reward') is not None:
                act['aux1'] = float(k['failed_dropoff_reward'])
        out.append(act)
    return out


def compile_spec(config_path, custom_level_path: Optional[str] = None, custom_modules_path: Optional[str] = None) -> EnvSpec:
    config_path = Path(config_path)
    if not config_path.exists() and (CONFIGS_DIR / config_path.name).exists():
        config_path = CONFIGS_DIR / config_path.name
    with open(config_path) as f:
        cfg = yaml.safe_load(f)
    gen = cfg['General']
    if not gen.get('individual_rewards', True):
        # Q26: with individual_rewards false the reference's Factory.step always raises (factory.py:217 sums the
        # float that summarize_step_results returns, :256-259), so that mode has no behaviour to reproduce
        raise UnsupportedSpec('individual_rewards: false crashes Factory.step in the reference (Q26, '
                              'environment/factory.py:217); only individual rewards are supported')
    level_name = gen['level_name']
    lvl = Path(custom_level_path) if custom_level_path else LEVELS_DIR / f'{level_name}.txt'
    H, W, level, floor, walls, doors = _parse_level(lvl)
    pomdp_r = int(gen['pomdp_r'])
    if pomdp_r < 0:
        raise UnsupportedSpec('pomdp_r must be >= 0')
    # the ray radius is the window diameter (Q13), so a ray has 2 * pomdp_r + 2 points (min(H, W) + 1 with full
    # observability); rays of up to 64 points render from registers (one 64-bit point mask), longer ones (up to 255
    # points) on the long-ray render (k_obs_lr: 32-point segments, per-agent tables in HBM)
    if pomdp_r > 126:
        raise UnsupportedSpec('pomdp_r is limited to 126 (rays of <= 255 points)')
    if pomdp_r == 0 and min(H, W) > 254:
        raise UnsupportedSpec('full observability (pomdp_r 0) is limited to levels with min(H, W) <= 254')
    d = 2 * pomdp_r + 1
    size = pomdp_r ** 2 if pomdp_r else H * W  # LevelParser.size (level_parser.py:44), collection cap (Q16)

    # ---- entities (config_parser.py:80-126), YAML order ----
    ents = cfg.get('Entities') or {}
    group_names = []
    for name in ents:
        if name == 'Defaults':  # FactoryConfigParser.default_entites is empty (config_parser.py:17,83-85)
            continue
        if name not in _GROUPS:
            raise UnsupportedSpec(f'entity group {name!r} is not implemented by the engine')
        group_names.append(name)
    ekw = {k: (v or {}) for k, v in ents.items() if k != 'Defaults'}
    if 'Doors' in ekw and not len(doors):
        raise UnsupportedSpec('Doors requires a D in the level (level_parser.py:96-98)')

    # ---- agents (config_parser.py:128-199) ----
    agents_conf = cfg['Agents']
    agent_names, agent_actions, agent_obs, agent_blocking, agent_positions = [], [], [], [], []
    for name, ac in agents_conf.items():
        positions = _literal_cells(ac.get('Positions') or [], H, W, f'Agents.{name}.Positions')
        acts = _parse_actions(ac['Actions'])
        obs = []
        if ac.get('Observations') is None:
            raise UnsupportedSpec('Did you specify any Observation?')
        if 'Defaults' in ac['Observations']:
            obs += ['Walls', 'Agent']
        obs += [x for x in ac['Observations'] if x != 'Defaults']
        other = {k: v for k, v in ac.items() if k not in ('Actions', 'Observations', 'Positions', 'Clones')}
        unknown = set(other) - {'is_blocking_pos'}
        if unknown:
            raise UnsupportedSpec(f'unknown agent kwargs {unknown}')
        blocking = bool(other.get('is_blocking_pos', False))
        names = [name]
        clones = ac.get('Clones', 0)
        if clones:
            if isinstance(clones, int):
                clones = [f'{name}_the_{n}{_n_abbr(n)}' for n in range(clones)]
            names += list(clones)
        for n in names:  # clones share the conf, Positions included (config_parser.py:189-194)
            agent_names.append(n)
            agent_actions.append(acts)
            agent_obs.append(obs)
            agent_blocking.append(blocking)
            agent_positions.append(positions)
    A = len(agent_names)
    if A > abi.MAX_AGENTS:
        raise UnsupportedSpec(f'{A} agents > {abi.MAX_AGENTS}')
    full = [f'Agent[{n}]' for n in agent_names]

    # ---- observation layers (observation_builder.py:237-277 + build_for_agent resolution :164-220) ----
    layer_names, layer_prog, combined = [], [], []
    for i, obs in enumerate(agent_obs):
        me = full[i]
        names, prog, comb = [], [], None
        for o in obs:
            vals = None
            if isinstance(o, dict):
                o, vals = next(iter(o.items()))
            if o == 'Self':
                names.append(me)
            elif o == 'Combined':
                if isinstance(vals, str):
                    vals = [vals]
                members = []
                for v in vals:
                    if v == 'Self':
                        members.append(me)
                    elif v == 'Other':
                        members += [x for x in full if x != me]
                    else:
                        members.append(v)
                comb = members  # the last Combined wins: all_obs['Combined(<agent>)'] (Q: same key)
                names.append(f'Combined({me})')
            elif o == 'Other':
                names += [x for x in full if x != me]
            elif o == 'Agent':
                names += list(full)
            else:
                names.append(o)
        for ln in names:
            if ln.startswith('Combined('):
                prog.append((abi.LAYER_COMBINED, 0))
            elif ln == 'Placeholder':
                prog.append((abi.LAYER_ZERO, 0))
            elif ln in full:
                prog.append((abi.LAYER_TAG, abi.TAG_AGENT0 + full.index(ln)))
            elif ln in _POS_TAGS and (ln == 'Walls' or ln in group_names):
                prog.append((abi.LAYER_TAG, _POS_TAGS[ln]))
            elif ln == 'Battery' and 'Batteries' in group_names:
                prog.append((abi.LAYER_BATTERY, 0))
            elif ln == 'GlobalPosition' and 'GlobalPositions' in group_names:
                prog.append((abi.LAYER_GLOBALPOS, 0))
            elif ln == 'Inventory' and 'Inventories' in group_names:
                prog.append((abi.LAYER_ZERO, 0))  # positional Inventory collection: skipped (Q8)
            elif ln == 'Destination' and 'Destinations' in group_names:
                prog.append((abi.LAYER_ZERO, 0))  # regex-bound positional destination: skipped
            else:
                raise UnsupportedSpec(f'observation layer {ln!r} of {me} cannot be resolved (exit upstream)')
        ctags = []
        for m in (comb or []):
            if m in full:
                ctags.append(abi.TAG_AGENT0 + full.index(m))
            elif m in _POS_TAGS:
                ctags.append(_POS_TAGS[m])
        if len(prog) > abi.MAX_LAYERS:
            raise UnsupportedSpec('too many observation layers')
        layer_names.append(names)
        layer_prog.append(prog)
        combined.append(ctags)

    # ---- rules (config_parser.py:201-274; factory.py:117-119) ----
    rules_conf = cfg.get('Rules') or {}
    if 'Defaults' in rules_conf:
        raise UnsupportedSpec("Rules: Defaults loads 'WatchCollision' and exits upstream (Q23)")
    rules, rule_names = [], []
    host_rules = []  # custom rules (custom_modules_path) run on the host: (slot, name, class, kwargs)
    battery_cost_dict = None
    dest_entries = []
    for rname, rkw in rules_conf.items():
        rkw = rkw or {}
        if rname not in _RULES:
            # config_parser.py:218-233: built-in folders first, then the custom path
            cls = None
            if custom_modules_path is not None:
                from .host_rules import locate_custom_class
                cls = locate_custom_class(rname, custom_modules_path)
            if cls is None:
                raise UnsupportedSpec(f'rule {rname!r} is not implemented by the engine'
                                      + (f' and not found in {custom_modules_path}' if custom_modules_path else ''))
            host_rules.append((len(rules), rname, cls, rkw))
            continue
        op = _RULES[rname]
        ri, rf = [0] * 6, [0.0] * 6
        if op == abi.RULE_DOOR_AUTOCLOSE:
            if 'Doors' not in group_names:
                raise UnsupportedSpec('DoorAutoClose without Doors inserts None into Entities (Q15)')
        elif op == abi.RULE_RESPAWN_ITEMS:
            ri[0] = int(rkw.get('n_items', 5))
            ri[1] = int(rkw.get('respawn_freq', 15))
        elif op == abi.RULE_WATCH_COLLISIONS:
            rf[0] = float(rkw.get('reward', -0.5))
            ri[0] = int(bool(rkw.get('done_at_collisions', False)))
            rf[1] = float(rkw.get('reward_at_done', -1))
        elif op in (abi.RULE_BATTERY_DECHARGE, abi.RULE_DONE_BATTERY):
            cost = rkw.get('per_action_costs', 0.02)
            if isinstance(cost, dict):
                # energy_consumption = per_action_costs[agent.state.identifier] (batteries/rules.py:54-58): keyed
                # by the ActionResult identifier = the action's class name; a paralyzed agent's state is 'Noop'
                cost = {str(k): float(v) for k, v in cost.items()}
                if battery_cost_dict is not None and battery_cost_dict != cost:
                    raise UnsupportedSpec('two battery rules with different per_action_costs dicts')
                battery_cost_dict = cost
                ri[2] = 1
                ri[3] = int('Noop' in cost)
                rf[3] = cost.get('Noop', 0.0)
            else:
                rf[0] = float(cost)
            rf[1] = float(rkw.get('battery_discharge_reward', -1.0))
            ri[0] = int(bool(rkw.get('paralyze_agents_on_discharge', False)))
            if op == abi.RULE_DONE_BATTERY:
                ri[1] = int(rkw.get('mode', 'grouped') == 'grouped')  # b.SINGLE == "grouped" (Q10)
                rf[2] = float(rkw.get('reward_discharge_done', -1.0))
            if 'Batteries' not in group_names:
                raise UnsupportedSpec(f'{rname} without Batteries')
        elif op == abi.RULE_DONE_MAXSTEPS:
            ri[0] = int(rkw.get('max_steps', 500))
        elif op == abi.RULE_RESPAWN_DIRT:
            ri[0] = int(rkw.get('respawn_freq', 15))
            ri[1] = int(rkw.get('respawn_n', 5))
            rf[0] = float(rkw.get('respawn_amount', 1.0))
        elif op == abi.RULE_DONE_DIRT:
            rf[0] = float(rkw.get('reward', 4.5))
        elif op == abi.RULE_DONE_MAINT_COLLISION:
            rf[0] = -5.0  # maintenance/constants.py MAINTAINER_COLLISION_REWARD (the rule takes no kwargs)
        elif op == abi.RULE_DEST_REACH:
            rf[0] = float(rkw.get('dest_reach_reward', 1.0))
        elif op == abi.RULE_DONE_DEST:
            rf[0] = float(rkw.get('dest_reach_reward', 1.0))
            rf[1] = float(rkw.get('reward_at_done', 5.0))
            ri[0] = {'any': abi.DEST_ANY, 'all': abi.DEST_ALL, 'simultaneous': abi.DEST_SIMULTANEOUS}[
                rkw.get('condition', 'any')]
        elif op == abi.RULE_RANDOM_INIT_STEPS:
            if 'random_steps' not in rkw:  # `def __init__(self, random_steps: 10)` has no default (rules.py:329)
                raise UnsupportedSpec('DoRandomInitialSteps needs random_steps (TypeError upstream)')
            ri[0] = int(rkw['random_steps'])
        rules.append((op, ri, rf))
        rule_names.append(rname)
    # spawn rules in Entities order (Walls, Agents have none)
    for g in group_names:
        kw = ekw[g]
        op = _GROUPS[g][1]
        if op is None:
            continue
        if kw.get('spawnrule'):  # Collection.spawn_rule (collection.py:66-77): the given rule replaces SpawnEntity
            if g != 'Destinations':
                raise UnsupportedSpec(f'{g}: spawnrule is only implemented for Destinations')
            for sr_name, sr_kw in kw['spawnrule'].items():
                if sr_name not in _DEST_SPAWNRULES:
                    raise UnsupportedSpec(f'spawnrule {sr_name!r} is not implemented by the engine')
                sr_kw = sr_kw or {}
                if sr_name == 'SpawnDestinationsPerAgent':
                    if set(sr_kw) != {'coords_or_quantity'} or not isinstance(sr_kw['coords_or_quantity'], dict):
                        raise UnsupportedSpec('SpawnDestinationsPerAgent takes coords_or_quantity: {agent: [...]}')
                    for an, val in sr_kw['coords_or_quantity'].items():
                        # agent = get_first(state[AGENT], lambda x: agent_name in x.name) (rules.py:114)
                        hit = [i for i, n in enumerate(agent_names) if str(an) in f'Agent[{n}]']
                        if not hit:
                            raise UnsupportedSpec(f'SpawnDestinationsPerAgent: no agent matches {an!r} (assert upstream)')
                        if isinstance(val, int):
                            dest_entries.append((hit[0], val, []))
                        else:
                            dest_entries.append((hit[0], 0, _literal_cells(val, H, W, f'destinations of {an}')))
                elif sr_kw:
                    raise UnsupportedSpec(f'{sr_name} takes no kwargs')
                rules.append((_DEST_SPAWNRULES[sr_name], [0] * 6, [0.0] * 6))
                rule_names.append(sr_name)
            continue
        ri, rf = [0] * 6, [0.0] * 6
        q = kw.get('coords_or_quantity')
        if op in (abi.RULE_SPAWN_PODS, abi.RULE_SPAWN_DROPOFFS, abi.RULE_SPAWN_ITEMS, abi.RULE_SPAWN_DESTS,
                  abi.RULE_SPAWN_MACHINES, abi.RULE_SPAWN_MAINTAINERS):
            if not isinstance(q, int) or q <= 0:
                raise UnsupportedSpec(f'{g}: coords_or_quantity must be a positive int (None crashes upstream)')
            ri[0] = q
            ri[1] = int(bool(kw.get('ignore_blocking', False)))
        rules.append((op, ri, rf))
        rule_names.append(f'SpawnEntity({g})')
    if len(rules) > abi.MAX_RULES:
        raise UnsupportedSpec('too many rules')
    if 'MoveMaintainers' in rules_conf and not {'Maintainers', 'Machines', 'Doors'} <= set(group_names):
        raise UnsupportedSpec('MoveMaintainers needs Maintainers, Machines and Doors (missing groups insert None, Q15)')
    if 'DoneAtMaintainerCollision' in rules_conf and 'Maintainers' not in group_names:
        raise UnsupportedSpec('DoneAtMaintainerCollision without Maintainers (Q15)')
    for g, cap_needed in (('Batteries', A), ('GlobalPositions', A)):
        if g in group_names and cap_needed > size + 1:
            raise UnsupportedSpec(f'{g}: {cap_needed} agents exceed LevelParser.size+1={size + 1} (Q16)')

    if len(dest_entries) > abi.MAX_AGENTS:
        raise UnsupportedSpec('too many SpawnDestinationsPerAgent entries')
    rays = ray_table(d if pomdp_r else min(H, W))  # RayCaster(agent, min(obs_shape)) (Q13)
    ray_off = np.zeros(len(rays) + 1, np.int32)
    ray_off[1:] = np.cumsum([len(r) for r in rays])
    ray_pts = np.asarray([p for r in rays for p in r], np.int32).reshape(-1)

    es = EnvSpec(config_path=str(config_path), level_name=level_name, H=H, W=W, level=level,
                 floor_cells=floor, wall_cells=walls, door_cells=doors, pomdp_r=pomdp_r,
                 ray_off=ray_off, ray_pts=ray_pts, agent_names=agent_names,
                 action_classes=[[a['cls'] for a in acts] for acts in agent_actions],
                 action_idents=[[a['ident'] for a in acts] for acts in agent_actions],
                 layer_names=layer_names, rule_names=rule_names, group_names=group_names,
                 individual_rewards=bool(gen.get('individual_rewards', True)),
                 env_seed=int(gen.get('env_seed', 69)))
    es.agent_actions = agent_actions
    es.layer_prog = layer_prog
    es.combined = combined
    es.rules = rules
    es.ekw = ekw
    es.agent_blocking = agent_blocking
    es.agent_positions = agent_positions
    es.battery_cost_dict = battery_cost_dict
    es.dest_entries = dest_entries
    es.host_rules = host_rules
    es.c = _to_c(es)
    return es


def _ptr(arr, ctype, keep):
    arr = np.ascontiguousarray(arr)
    keep.append(arr)
    return arr.ctypes.data_as(C.POINTER(ctype))


def _to_c(es: EnvSpec) -> abi.MfgSpec:
    s = abi.MfgSpec()
    k = es._keep
    s.abi_version = abi.ABI_VERSION
    s.H, s.W = es.H, es.W
    s.level = _ptr(es.level.astype(np.uint8), C.c_uint8, k)
    s.n_floor = len(es.floor_cells)
    s.floor_cells = _ptr(es.floor_cells.astype(np.int32), C.c_int32, k)
    s.n_walls = len(es.wall_cells)
    s.wall_cells = _ptr(es.wall_cells.astype(np.int32), C.c_int32, k)
    s.n_doors = len(es.door_cells) if 'Doors' in es.group_names else 0
    if s.n_doors > abi.MAX_DOORS:
        raise UnsupportedSpec('too many doors')
    s.door_cells = _ptr(es.door_cells.astype(np.int32), C.c_int32, k)
    dk = es.ekw.get('Doors', {}) if 'Doors' in es.group_names else {}
    s.door_closed_on_init = int(bool(dk.get('closed_on_init', True)))
    s.door_auto_close = int(dk.get('auto_close_interval', 10))
    s.pomdp_r = es.pomdp_r
    s.n_rays = len(es.ray_off) - 1
    s.ray_off = _ptr(es.ray_off, C.c_int32, k)
    s.ray_pts = _ptr(es.ray_pts, C.c_int32, k)
    s.n_agents = es.n_agents
    for a in range(es.n_agents):
        s.agent_blocking[a] = int(es.agent_blocking[a])
        s.n_positions[a] = len(es.agent_positions[a])
        for j, cell in enumerate(es.agent_positions[a]):
            s.positions[a][j] = cell
        acts = es.agent_actions[a]
        if len(acts) > abi.MAX_ACTIONS:
            raise UnsupportedSpec('too many actions')
        s.n_actions[a] = len(acts)
        for j, ac in enumerate(acts):
            s.actions[a][j].op = ac['op']
            s.actions[a][j].arg = ac['arg']
            s.actions[a][j].valid_reward = ac['valid']
            s.actions[a][j].fail_reward = ac['fail']
            s.actions[a][j].aux0 = ac['aux0']
            s.actions[a][j].aux1 = ac['aux1']
            bc = es.battery_cost_dict
            s.actions[a][j].battery_cost = (bc.get(ac['cls'], float('nan')) if bc is not None else 0.0)
        s.n_layers[a] = len(es.layer_prog[a])
        for j, (kind, tag) in enumerate(es.layer_prog[a]):
            s.layers[a][j].kind = kind
            s.layers[a][j].tag = tag
        if len(es.combined[a]) > abi.MAX_COMBINED:
            raise UnsupportedSpec(f'a Combined layer with more than {abi.MAX_COMBINED} members')
        s.combined_n[a] = len(es.combined[a])
        for j, t in enumerate(es.combined[a]):
            s.combined_tags[a][j] = t
    g = es.group_names
    ek = es.ekw
    s.has_batteries = int('Batteries' in g)
    s.battery_initial = float(ek.get('Batteries', {}).get('initial_charge_level', 1.0))
    s.has_inventories = int('Inventories' in g)
    s.has_items = int('Items' in g)
    s.items_quantity = int(ek.get('Items', {}).get('coords_or_quantity') or 0)
    s.has_pods = int('ChargePods' in g)
    s.pod_charge_rate = 0.4  # ChargePod(charge_rate=0.4): collection kwargs are not forwarded
    s.has_dropoffs = int('DropOffLocations' in g)
    s.has_dirt = int('DirtPiles' in g)
    dk = ek.get('DirtPiles', {})
    s.dirt_quantity = int(dk.get('coords_or_quantity', 10))
    s.dirt_initial_amount = float(dk.get('initial_amount', 2))
    s.dirt_clean_amount = float(dk.get('clean_amount', 1))
    s.dirt_max_global = float(dk.get('max_global_amount', 20))
    s.dirt_max_local = float(dk.get('max_local_amount', 5))
    s.dirt_amount_var = float(dk.get('amount_var', 0.2))
    s.dirt_n_var = float(dk.get('n_var', 0.2))
    s.has_dests = int('Destinations' in g)
    s.dest_action_counts = 0
    s.has_machines = int('Machines' in g)
    s.machine_work, s.machine_pause = 10, 15
    s.has_maintainers = int('Maintainers' in g)
    s.has_globalpos = int('GlobalPositions' in g)
    s.has_doors = int('Doors' in g)
    s.n_rules = len(es.rules)
    for j, (op, ri, rf) in enumerate(es.rules):
        s.rules[j].op = op
        for q in range(6):
            s.rules[j].i[q] = ri[q]
            s.rules[j].f[q] = rf[q]
    s.n_dest_entries = len(es.dest_entries)
    for j, (agent, q, cells) in enumerate(es.dest_entries):
        s.dest_entry_agent[j] = agent
        s.dest_entry_q[j] = q
        s.dest_entry_n[j] = len(cells)
        for k, cell in enumerate(cells):
            s.dest_entry_cells[j][k] = cell
    s.individual_rewards = int(es.individual_rewards)
    s.env_seed = es.env_seed & 0xFFFFFFFF
    return s


def seed_key(py_seed: int) -> np.ndarray:
    """random.seed(int): init_by_array over the 32-bit little-endian chunks of abs(seed) (_randommodule.c)."""
    n = abs(int(py_seed))
    words = []
    while True:
        words.append(n & 0xFFFFFFFF)
        n >>= 32
        if not n:
            break
    return np.asarray(words, np.uint32)

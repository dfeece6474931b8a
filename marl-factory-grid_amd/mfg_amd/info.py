"""Host-side rebuild of the reference's per-step Result list from the engine's event record.

The reference walks the ordered Result list of a step (factory.py:222-259, utils/results.py:42-84):
* `info`: key '<entity.name or Global>_<identifier>' accumulates reward, then value, in result order;
  ActionResults add '<agent>_Collisions': 1 when the action introduced a collision; `step_reward` and
  `step` are appended;
* `reward`: per entity name the f64 sum of the results' rewards in result order; an individual reward is
  the agent's sum + the sum of the entity-less ('global') results (factory.py:245-253).
The engine emits a compact `MfgEvents` record per env-step instead of Python objects. `step_results`
replays the same ordered list on the host (pre-step, agent actions, tick_step, tick_post_step and
check_done results in rule order); `rebuild_info` / `rebuild_rewards` fold it exactly like the reference,
so a B=1 `Factory` returns the identical dict and, with host-side custom rules merged into the list
(mfg_amd/host_rules.py), the identical rewards.
"""
from collections import defaultdict
from dataclasses import dataclass
from typing import Optional

from . import abi

# result phases in Gamestate.tick / check_done order (states.py:170-226)
PRE, ACT, TICK, POST, DONE = range(5)


@dataclass
class Res:
    """One reference Result: entity name (None = Global), agent index of the entity (-1 = not an agent),
    identifier, reward / value (None = absent), the ActionResult collision flag, validity."""
    entity: Optional[str]
    agent: int
    ident: str
    reward: Optional[float] = None
    value: Optional[float] = None
    collision: bool = False
    valid: bool = True
    phase: int = TICK
    slot: int = 0  # device rule index (results of one phase come in rule order)


def step_results(spec, actions, ev):
    """The device step's Result list in reference order. spec: EnvSpec; actions: per-agent ints;
    ev: MfgEvents (or a dict with the same fields)."""
    g = (lambda k: ev[k]) if isinstance(ev, dict) else (lambda k: getattr(ev, k))
    out = []
    names = [f'Agent[{n}]' for n in spec.agent_names]
    act = g('act')
    watch = g('watch')
    # 1) agent action results (states.py:187-196)
    for a, n in enumerate(names):
        bits = act[a]
        if not bits & 0x80:
            continue
        ac = spec.agent_actions[a][int(actions[a])]
        if bits & 4:  # ItemAction drop-off branch (items/actions.py:43-52)
            r = ac['aux0'] if bits & 1 else ac['aux1']
        else:
            r = ac['valid'] if bits & 1 else ac['fail']
        out.append(Res(n, a, ac['cls'], reward=r, collision=bool(bits & 2), valid=bool(bits & 1), phase=ACT, slot=-1))
    # 2) tick_step results in rule order
    dest_count = [(w >> 3) & 31 for w in watch]  # destinations credited per agent (ev_watch bits 3..7)
    for ri, (op, ri_, rf) in enumerate(spec.rules):
        rname = spec.rule_names[ri]
        if op == abi.RULE_DOOR_AUTOCLOSE and g('door_autoclose'):
            out.append(Res(None, -1, rname, value=1, phase=TICK, slot=ri))
        elif op in (abi.RULE_BATTERY_DECHARGE, abi.RULE_DONE_BATTERY):
            for a, n in enumerate(names):
                if ri_[2]:  # per_action_costs[agent.state.identifier]: the action's class, 'Noop' if paralyzed
                    cls = spec.agent_actions[a][int(actions[a])]['cls'] if act[a] & 0x80 else 'Noop'
                    v = spec.battery_cost_dict[cls]
                else:
                    v = rf[0]
                out.append(Res(n, a, rname, value=v, phase=TICK, slot=ri))
        elif op == abi.RULE_RESPAWN_DIRT and g('dirt_spawn_value') >= 0:
            out.append(Res(None, -1, 'DirtPiles_spawn', value=g('dirt_spawn_value'), valid=bool(g('dirt_spawn_valid')),
                           phase=TICK, slot=ri))
        elif op in (abi.RULE_DEST_REACH, abi.RULE_DONE_DEST):
            for a, n in enumerate(names):
                for _ in range(dest_count[a]):
                    out.append(Res(n, a, rname, reward=rf[0], phase=TICK, slot=ri))
            dest_count = [0] * len(names)  # a second reach rule sees every destination already marked
    # 3) tick_post_step results in rule order
    for ri, (op, ri_, rf) in enumerate(spec.rules):
        rname = spec.rule_names[ri]
        if op == abi.RULE_RESPAWN_ITEMS and g('respawn_items_value') >= 0:
            out.append(Res(None, -1, rname, value=g('respawn_items_value'), phase=POST, slot=ri))
        elif op == abi.RULE_WATCH_COLLISIONS:
            for a, n in enumerate(names):
                if watch[a] & 1:
                    out.append(Res(n, a, 'Collisions', reward=rf[0], valid=False, phase=POST, slot=ri))
            dc, d = int(g('door_coll')) | (int(g('door_coll_hi')) << 64), 0  # doors 0..127
            while dc:
                if dc & 1:
                    out.append(Res(f'Door[{d}]', -1, 'Collisions', reward=rf[0], valid=False, phase=POST, slot=ri))
                dc >>= 1
                d += 1
            mc, k = int(g('maint_coll')), 0
            while mc:  # maintainers of one SpawnEntity call have consecutive u_ints
                if mc & 1:
                    out.append(Res(f"Maintainer[{int(g('maint_base')) + k}]", -1, 'Collisions', reward=rf[0],
                                   valid=False, phase=POST, slot=ri))
                mc >>= 1
                k += 1
        elif op in (abi.RULE_BATTERY_DECHARGE, abi.RULE_DONE_BATTERY):
            for a, n in enumerate(names):
                if watch[a] & 2:
                    out.append(Res(n, a, rname, reward=rf[1], phase=POST, slot=ri))
    # 4) done results in rule order (states.py:216-226); WatchCollisions' DoneResult (done_mask bit 31) sits at
    # its own rule position, so the global f64 sum sees it in the reference's order
    dm = int(g('done_mask'))
    for ri, (op, ri_, rf) in enumerate(spec.rules):
        rname = spec.rule_names[ri]
        if op == abi.RULE_WATCH_COLLISIONS:
            if dm & (1 << 31):
                out.append(Res(None, -1, 'Collisions', reward=rf[1], phase=DONE, slot=ri))
            continue
        if not dm & (1 << ri):
            continue
        if op == abi.RULE_DONE_BATTERY:
            out.append(Res(None, -1, rname, reward=rf[2], phase=DONE, slot=ri))
        elif op == abi.RULE_DONE_DIRT:
            out.append(Res(None, -1, rname, reward=rf[0], phase=DONE, slot=ri))
        elif op == abi.RULE_DONE_DEST:
            out.append(Res(None, -1, rname, reward=rf[1], phase=DONE, slot=ri))
        elif op == abi.RULE_DONE_MAINT_COLLISION:  # one DoneResult per agent standing on a maintainer
            for a, n in enumerate(names):
                if watch[a] & 4:
                    out.append(Res(n, a, rname, reward=rf[0], phase=DONE, slot=ri))
        else:
            out.append(Res(None, -1, rname, phase=DONE, slot=ri))
    return out


def fold_info(results):
    """utils/results.py:42-84 + factory.py:231-240: the info dict of an ordered Result list."""
    info = defaultdict(float)
    for r in results:
        key = f"{r.entity if r.entity is not None else 'Global'}_{r.ident}"
        if r.reward is not None:
            info[key] += r.reward
        if r.value is not None:
            info[key] += r.value
        if r.collision:
            info[f'{r.entity}_Collisions'] += 1
    return info


def rebuild_rewards(spec, results):
    """factory.py:230-253: per-agent f64 reward sums in result order, plus the global sum."""
    own = [0.0] * spec.n_agents
    glob = 0.0
    for r in results:
        if r.reward is None:
            continue
        if r.entity is None:
            glob += r.reward
        elif r.agent >= 0:
            own[r.agent] += r.reward
    return [x + glob for x in own]


def rebuild_info(spec, actions, ev, reward, results=None):
    """The reference info dict of one step (results: a precomputed/merged Result list, else the device's)."""
    res = step_results(spec, actions, ev) if results is None else results
    out = dict(fold_info(res))
    out['step_reward'] = sum(reward)
    g = (lambda k: ev[k]) if isinstance(ev, dict) else (lambda k: getattr(ev, k))
    out['step'] = g('step')
    return out

"""Host-side rebuild of the reference info dict from the engine's per-step event record.

The reference builds `info` by walking the ordered Result list of a step (factory.py:222-259,
utils/results.py:42-84): key '<entity.name or Global>_<identifier>' accumulates reward and value in
result order, ActionResults add '<agent>_Collisions': 1 when the action introduced a collision, then
`step_reward=sum(reward)` and `step` are appended. The engine emits a compact `MfgEvents` record per
env-step instead of Python objects; this module replays the same result order on the host so a B=1
`Factory` facade returns the identical dict.
"""
from collections import defaultdict

from . import abi


def rebuild_info(spec, actions, ev, reward):
    """spec: EnvSpec; actions: per-agent ints; ev: MfgEvents (or a dict with the same fields); reward: list."""
    g = (lambda k: ev[k]) if isinstance(ev, dict) else (lambda k: getattr(ev, k))
    info = defaultdict(float)
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
            info[f"{n}_{ac['cls']}"] += ac['aux0'] if bits & 1 else ac['aux1']
        else:
            info[f"{n}_{ac['cls']}"] += ac['valid'] if bits & 1 else ac['fail']
        if bits & 2:
            info[f'{n}_Collisions'] += 1
    # 2) tick_step results in rule order
    dest_count = [(w >> 3) & 31 for w in watch]  # destinations credited per agent (ev_watch bits 3..7)
    for ri, (op, ri_, rf) in enumerate(spec.rules):
        rname = spec.rule_names[ri]
        if op == abi.RULE_DOOR_AUTOCLOSE and g('door_autoclose'):
            info[f'Global_{rname}'] += 1
        elif op in (abi.RULE_BATTERY_DECHARGE, abi.RULE_DONE_BATTERY):
            for a, n in enumerate(names):
                if ri_[2]:  # per_action_costs[agent.state.identifier]: the action's class, 'Noop' if paralyzed
                    cls = spec.agent_actions[a][int(actions[a])]['cls'] if act[a] & 0x80 else 'Noop'
                    info[f'{n}_{rname}'] += spec.battery_cost_dict[cls]
                else:
                    info[f'{n}_{rname}'] += rf[0]
        elif op == abi.RULE_RESPAWN_DIRT and g('dirt_spawn_value') >= 0:
            info['Global_DirtPiles_spawn'] += g('dirt_spawn_value')
        elif op in (abi.RULE_DEST_REACH, abi.RULE_DONE_DEST):
            for a, n in enumerate(names):
                for _ in range(dest_count[a]):
                    info[f'{n}_{rname}'] += rf[0]
            dest_count = [0] * len(names)  # a second reach rule sees every destination already marked
    # 3) tick_post_step results in rule order
    for ri, (op, ri_, rf) in enumerate(spec.rules):
        rname = spec.rule_names[ri]
        if op == abi.RULE_RESPAWN_ITEMS and g('respawn_items_value') >= 0:
            info[f'Global_{rname}'] += g('respawn_items_value')
        elif op == abi.RULE_WATCH_COLLISIONS:
            for a, n in enumerate(names):
                if watch[a] & 1:
                    info[f'{n}_Collisions'] += rf[0]
            dc = int(g('door_coll'))
            d = 0
            while dc:
                if dc & 1:
                    info[f'Door[{d}]_Collisions'] += rf[0]
                dc >>= 1
                d += 1
            mc, k = int(g('maint_coll')), 0
            while mc:  # maintainers of one SpawnEntity call have consecutive u_ints
                if mc & 1:
                    info[f"Maintainer[{int(g('maint_base')) + k}]_Collisions"] += rf[0]
                mc >>= 1
                k += 1
        elif op in (abi.RULE_BATTERY_DECHARGE, abi.RULE_DONE_BATTERY):
            for a, n in enumerate(names):
                if watch[a] & 2:
                    info[f'{n}_{rname}'] += rf[1]
    # 4) done results (states.py:216-226)
    dm = int(g('done_mask'))
    for ri, (op, ri_, rf) in enumerate(spec.rules):
        if not dm & (1 << ri):
            continue
        rname = spec.rule_names[ri]
        if op == abi.RULE_DONE_BATTERY:
            info[f'Global_{rname}'] += rf[2]
        elif op in (abi.RULE_DONE_DIRT,):
            info[f'Global_{rname}'] += rf[0]
        elif op == abi.RULE_DONE_DEST:
            info[f'Global_{rname}'] += rf[1]
        elif op == abi.RULE_DONE_MAINT_COLLISION:  # one DoneResult per agent standing on a maintainer
            for a, n in enumerate(names):
                if watch[a] & 4:
                    info[f'{n}_{rname}'] += rf[0]
    if dm & (1 << 31):
        for op, ri_, rf in spec.rules:
            if op == abi.RULE_WATCH_COLLISIONS:
                info['Global_Collisions'] += rf[1]
    out = dict(info)
    out['step_reward'] = sum(reward)
    out['step'] = g('step')
    return out

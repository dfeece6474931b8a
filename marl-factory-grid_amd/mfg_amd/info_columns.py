"""Batched info: the reference's per-step info dict as device columns for all B envs.

`Factory.step` returns `info`, a dict built by `summarize_step_results` (environment/factory.py:222-259):
key '<entity.name or Global>_<identifier>' accumulates each Result's reward and value in result order
(utils/results.py:42-52), ActionResults add '<agent>_Collisions': 1 (results.py:62-84), then
`step_reward = sum(reward)` and `step` are set. `info.rebuild_info` rebuilds that dict for ONE env on the host.
For B >> 1 this module evaluates the same accumulation as torch ops over the batch, straight from the engine's
event rows (no host copy):

    cols = InfoColumns(spec)                       # the key set of this config, fixed at construction
    values, present = cols(actions, ev_act, ev_watch, ev_misc, reward)   # f64 [B, K], bool [B, K]
    cols.to_dict(values, present, b)               # == rebuild_info(...) of env b (tests/test_info_columns.py)

`present[b, k]` says whether key k is in env b's dict this step (a key with value 0.0 is still present, as in
the reference's defaultdict). Every value is accumulated in the reference's order, so the f64 sums are the
reference's bits. Maintainer collision keys depend on per-episode u_ints: they are columns per maintainer
slot; to_dict names them with the step's MFG_EVM_MAINT_BASE.
"""
from . import abi


class InfoColumns:
    def __init__(self, spec):
        self.spec = spec
        self.keys = []
        self._kidx = {}
        self._ops = []  # (key index, kind, params) in rebuild_info's accumulation order
        names = [f'Agent[{n}]' for n in spec.agent_names]
        A = len(names)
        self.A = A

        def key(k):
            if k not in self._kidx:
                self._kidx[k] = len(self.keys)
                self.keys.append(k)
            return self._kidx[k]

        # 1) agent action results (utils/states.py:187-196)
        for a, n in enumerate(names):
            classes = []
            for ac in spec.agent_actions[a]:
                if ac['cls'] not in classes:
                    classes.append(ac['cls'])
            for cls in classes:
                slots = [j for j, ac in enumerate(spec.agent_actions[a]) if ac['cls'] == cls]
                self._ops.append((key(f'{n}_{cls}'), 'action', (a, slots)))
            self._ops.append((key(f'{n}_Collisions'), 'act_coll', (a,)))
        # destination slots of one env (the engine's destmax, mfg_create): bounds the per-step reach count, so the
        # exact one-add-per-destination fold needs no device->host read of the count
        self._dest_max = 0
        for op, ri_, _ in spec.rules:
            if op == abi.RULE_SPAWN_DESTS:
                self._dest_max = int(ri_[0])
            elif op == abi.RULE_SPAWN_DEST_ON_AGENT:
                self._dest_max = spec.n_agents
            elif op == abi.RULE_SPAWN_DEST_PER_AGENT:
                self._dest_max = int(spec.c.n_dest_entries)
        self._dest_max = min(self._dest_max, 31)  # the 5-bit reach counter of ev_watch
        # 2) tick_step results in rule order
        dest_seen = False
        for ri, (op, ri_, rf) in enumerate(spec.rules):
            rname = spec.rule_names[ri]
            if op == abi.RULE_DOOR_AUTOCLOSE:
                self._ops.append((key(f'Global_{rname}'), 'door_autoclose', ()))
            elif op in (abi.RULE_BATTERY_DECHARGE, abi.RULE_DONE_BATTERY):
                for a, n in enumerate(names):
                    self._ops.append((key(f'{n}_{rname}'), 'battery_cost', (a, ri)))
            elif op == abi.RULE_RESPAWN_DIRT:
                self._ops.append((key('Global_DirtPiles_spawn'), 'dirt_spawn', ()))
            elif op in (abi.RULE_DEST_REACH, abi.RULE_DONE_DEST) and not dest_seen:
                dest_seen = True  # a second reach rule sees every destination already marked
                for a, n in enumerate(names):
                    self._ops.append((key(f'{n}_{rname}'), 'dest_reach', (a, rf[0])))
        # 3) tick_post_step results in rule order
        for ri, (op, ri_, rf) in enumerate(spec.rules):
            rname = spec.rule_names[ri]
            if op == abi.RULE_RESPAWN_ITEMS:
                self._ops.append((key(f'Global_{rname}'), 'respawn_items', ()))
            elif op == abi.RULE_WATCH_COLLISIONS:
                for a, n in enumerate(names):
                    self._ops.append((key(f'{n}_Collisions'), 'watch_bit', (a, 1, rf[0])))
                for d in range(spec.c.n_doors):
                    self._ops.append((key(f'Door[{d}]_Collisions'), 'door_coll', (d, rf[0])))
                kmax = next((r[1][0] for r in spec.rules if r[0] == abi.RULE_SPAWN_MAINTAINERS), 0)
                for k in range(kmax):
                    self._ops.append((key(f'Maintainer[slot {k}]_Collisions'), 'maint_coll', (k, rf[0])))
            elif op in (abi.RULE_BATTERY_DECHARGE, abi.RULE_DONE_BATTERY):
                for a, n in enumerate(names):
                    self._ops.append((key(f'{n}_{rname}'), 'watch_bit', (a, 2, rf[1])))
        # 4) done results (utils/states.py:216-226)
        for ri, (op, ri_, rf) in enumerate(spec.rules):
            rname = spec.rule_names[ri]
            if op == abi.RULE_DONE_BATTERY:
                self._ops.append((key(f'Global_{rname}'), 'done_bit', (ri, rf[2])))
            elif op == abi.RULE_DONE_DIRT:
                self._ops.append((key(f'Global_{rname}'), 'done_bit', (ri, rf[0])))
            elif op == abi.RULE_DONE_DEST:
                self._ops.append((key(f'Global_{rname}'), 'done_bit', (ri, rf[1])))
            elif op == abi.RULE_DONE_MAINT_COLLISION:
                for a, n in enumerate(names):
                    self._ops.append((key(f'{n}_{rname}'), 'maint_done', (a, ri, rf[0])))
        for op, ri_, rf in spec.rules:
            if op == abi.RULE_WATCH_COLLISIONS:
                self._ops.append((key('Global_Collisions'), 'done_bit', (31, rf[1])))
        self.n_keys = len(self.keys)

    def __call__(self, actions, ev_act, ev_watch, ev_misc, reward):
        """actions int [B, A], ev_act/ev_watch u8 [B, A], ev_misc i32 [B, MFG_EV_MISC_N], reward f64 [B, A]
        (all on one device) -> (values f64 [B, K + 2], present bool [B, K + 2]); the last two columns are
        'step_reward' and 'step' (always present)."""
        import torch
        B, dev = reward.shape[0], reward.device
        spec = self.spec
        f64 = torch.float64
        vals = torch.zeros((B, self.n_keys + 2), dtype=f64, device=dev)
        pres = torch.zeros((B, self.n_keys + 2), dtype=torch.bool, device=dev)
        act = ev_act.to(torch.int32)
        watch = ev_watch.to(torch.int32)
        misc = ev_misc.to(torch.int64)
        acts = actions.to(dev).to(torch.int64)
        acted = (act & 0x80) != 0
        flags = misc[:, abi.EVM_FLAGS]
        dmask = misc[:, abi.EVM_DONE_MASK] & 0xFFFFFFFF
        # per-agent reward tables of the action results: value by slot (drop-off branch: aux0 / aux1)
        tabs = {}

        def add(k, mask, v):
            v = v if isinstance(v, torch.Tensor) else torch.full((B,), float(v), dtype=f64, device=dev)
            vals[:, k] = torch.where(mask, vals[:, k] + v, vals[:, k])
            pres[:, k] |= mask

        for k, kind, p in self._ops:
            if kind == 'action':
                a, slots = p
                if a not in tabs:
                    acs = spec.agent_actions[a]
                    tabs[a] = tuple(torch.tensor([ac[f] for ac in acs], dtype=f64, device=dev)
                                    for f in ('valid', 'fail', 'aux0', 'aux1'))
                valid_t, fail_t, aux0_t, aux1_t = tabs[a]
                s = acts[:, a].clamp(0, len(spec.agent_actions[a]) - 1)
                ok = (act[:, a] & 1) != 0
                drop = (act[:, a] & 4) != 0
                v = torch.where(drop, torch.where(ok, aux0_t[s], aux1_t[s]), torch.where(ok, valid_t[s], fail_t[s]))
                mine = acted[:, a] & torch.isin(s, torch.tensor(slots, device=dev))
                add(k, mine, v)
            elif kind == 'act_coll':
                add(k, acted[:, p[0]] & ((act[:, p[0]] & 2) != 0), 1.0)
            elif kind == 'door_autoclose':
                add(k, (flags & 1) != 0, 1.0)
            elif kind == 'battery_cost':
                a, ri = p
                _, ri_, rf = spec.rules[ri]
                if ri_[2]:
                    costs = torch.tensor([spec.battery_cost_dict.get(ac['cls'], float('nan'))
                                          for ac in spec.agent_actions[a]], dtype=f64, device=dev)
                    s = acts[:, a].clamp(0, len(spec.agent_actions[a]) - 1)
                    v = torch.where(acted[:, a], costs[s],
                                    torch.full((B,), spec.battery_cost_dict.get('Noop', float('nan')), dtype=f64,
                                               device=dev))
                else:
                    v = rf[0]
                add(k, torch.ones(B, dtype=torch.bool, device=dev), v)  # every agent, every step
            elif kind == 'dirt_spawn':
                v = misc[:, abi.EVM_DIRT_SPAWN]
                add(k, v >= 0, v.to(f64))
            elif kind == 'dest_reach':
                a, r = p
                n = (watch[:, a] >> 3) & 31
                for c in range(self._dest_max):  # one addition per credited destination (no host sync)
                    add(k, n > c, r)
            elif kind == 'respawn_items':
                v = misc[:, abi.EVM_RESPAWN_ITEMS]
                add(k, v >= 0, v.to(f64))
            elif kind == 'watch_bit':
                a, bit, r = p
                add(k, (watch[:, a] & bit) != 0, r)
            elif kind == 'door_coll':  # door d: bit d & 31 of the d >> 5-th door column
                d, r = p
                add(k, ((misc[:, abi.EVM_DOOR_COLS[d >> 5]] >> (d & 31)) & 1) != 0, r)
            elif kind == 'maint_coll':
                kk, r = p
                add(k, ((misc[:, abi.EVM_MAINT_COLS[kk >> 5]] >> (kk & 31)) & 1) != 0, r)
            elif kind == 'done_bit':
                bit, r = p
                add(k, ((dmask >> bit) & 1) != 0, r)
            elif kind == 'maint_done':
                a, ri, r = p
                add(k, (((dmask >> ri) & 1) != 0) & ((watch[:, a] & 4) != 0), r)
        s = torch.zeros(B, dtype=f64, device=dev)
        for a in range(self.A):  # sum(reward): left to right from 0
            s = s + reward[:, a]
        vals[:, -2] = s
        vals[:, -1] = misc[:, abi.EVM_STEP].to(f64)
        pres[:, -2:] = True
        return vals, pres

    @property
    def columns(self):
        return self.keys + ['step_reward', 'step']

    def to_dict(self, values, present, b, maint_base=None):
        """Env b's info dict (the reference's key names) from the columns."""
        v = values[b].cpu().tolist()
        p = present[b].cpu().tolist()
        out = {}
        for k, name in enumerate(self.columns):
            if not p[k]:
                continue
            if name.startswith('Maintainer[slot '):
                slot = int(name[len('Maintainer[slot '):name.index(']')])
                name = f'Maintainer[{int(maint_base) + slot}]_Collisions'
            out[name] = int(v[k]) if name == 'step' else v[k]
        return out

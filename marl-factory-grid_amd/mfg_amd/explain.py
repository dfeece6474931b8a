"""What this engine accepts in a config (the reference's ConfigExplainer, utils/tools.py:21-240).

The reference discovers classes reflectively and dumps their constructor kwargs. Here the catalogue is the
spec compiler's (mfg_amd/spec.py): every class name it maps onto an engine opcode, with the YAML kwargs it
reads and their defaults. `get_*` return dicts, `save_*` write YAML, `save_all` writes one overview file.
"""
from pathlib import Path

import yaml

from . import spec as _spec

# YAML kwargs the compiler reads per class, with the reference's defaults (constructor signatures upstream)
_RULE_KWARGS = {
    'DoorAutoClose': {'close_frequency': 10},
    'RespawnItems': {'n_items': 5, 'respawn_freq': 15},
    'WatchCollisions': {'reward': -0.5, 'done_at_collisions': False, 'reward_at_done': -1},
    'BatteryDecharge': {'initial_charge': 0.8, 'per_action_costs': 0.02, 'battery_discharge_reward': -1.0,
                        'paralyze_agents_on_discharge': False},
    'DoneAtBatteryDischarge': {'reward_discharge_done': -1.0, 'mode': 'grouped', 'per_action_costs': 0.02,
                               'battery_discharge_reward': -1.0, 'paralyze_agents_on_discharge': False},
    'DoneAtMaxStepsReached': {'max_steps': 500},
    'RespawnDirt': {'respawn_freq': 15, 'respawn_n': 5, 'respawn_amount': 1.0},
    'EntitiesSmearDirtOnMove': {'smear_ratio': 0.2},
    'DoneOnAllDirtCleaned': {'reward': 4.5},
    'DestinationReachReward': {'dest_reach_reward': 1.0},
    'DoneAtDestinationReach': {'condition': 'any', 'reward_at_done': 5.0, 'dest_reach_reward': 1.0},
    'MoveMaintainers': {},
    'DoneAtMaintainerCollision': {},
    'DoRandomInitialSteps': {'random_steps': 10},
    'SpawnDestinationOnAgent': {},
    'SpawnDestinationsPerAgent': {'coords_or_quantity': {'<agent name>': ['(x, y)', '...']}},
}
_ENTITY_KWARGS = {
    'Batteries': {'initial_charge_level': 1.0},
    'ChargePods': {'coords_or_quantity': 1, 'ignore_blocking': False},
    'Destinations': {'coords_or_quantity': 1, 'ignore_blocking': False,
                     'spawnrule': {'SpawnDestinationOnAgent': {}}},
    'DirtPiles': {'coords_or_quantity': 10, 'initial_amount': 2, 'clean_amount': 1, 'max_global_amount': 20,
                  'max_local_amount': 5, 'amount_var': 0.2, 'n_var': 0.2},
    'Doors': {'closed_on_init': True, 'auto_close_interval': 10},
    'DropOffLocations': {'coords_or_quantity': 1, 'ignore_blocking': False},
    'GlobalPositions': {},
    'Inventories': {},
    'Items': {'coords_or_quantity': 5, 'ignore_blocking': False},
    'Machines': {'coords_or_quantity': 1, 'ignore_blocking': False},
    'Maintainers': {'coords_or_quantity': 1, 'ignore_blocking': False},
}


def _custom_rules(folder):
    """{name: {kwarg: default or '!'}} of the Rule subclasses defined under `folder` (tools.py:43-58 explains a
    class by its and its bases' __init__ signatures). Custom Rules are the custom plugin kind this build runs
    (on the host, mfg_amd.host_rules); custom Actions and Entities are rejected by compile_spec."""
    import inspect
    from .host_rules import custom_modules
    out = {}
    for mod in custom_modules(folder):
        for key, obj in vars(mod).items():
            if key.startswith('_') or not inspect.isclass(obj) or obj.__module__ != mod.__name__:
                continue
            if not any(b.__name__ == 'Rule' for b in obj.__mro__[1:]):
                continue
            params = {}
            for cls in reversed(obj.__mro__[:-1]):
                try:
                    params.update(inspect.signature(cls).parameters)
                except (TypeError, ValueError):
                    pass
            out[key] = {k: (v.default if v.default is not inspect.Parameter.empty else '!')
                        for k, v in params.items() if k not in ('self', 'args', 'kwargs')}
    return out


class ConfigExplainer:
    def __init__(self, custom_path=None):
        # utils/tools.py:24-39: with a custom path, its modules' classes are explained beside the built-ins
        self.custom_path = Path(custom_path) if custom_path is not None else None

    def get_actions(self):
        acts = {k: {'valid_reward': v[3], 'fail_reward': v[4]} for k, v in _spec._ACTIONS.items()}
        acts.update({k: {'valid_reward': -0.001, 'fail_reward': -0.05} for k in _spec._MOVE_GROUPS})
        return acts

    def get_entities(self):
        return {k: dict(v) for k, v in _ENTITY_KWARGS.items()}

    @staticmethod
    def get_general_section():
        return {'General': {'env_seed': 69, 'individual_rewards': True, 'level_name': 'large', 'pomdp_r': 3,
                            'verbose': False, 'tests': False}}

    def get_agent_section(self):
        return {'Agents': {'ExampleAgent': {'Actions': sorted(self.get_actions()),
                                           'Observations': self.get_observations(),
                                           'Positions': ['(x, y)'], 'Clones': 0, 'is_blocking_pos': False}}}

    def get_rules(self):
        out = {k: dict(v) for k, v in _RULE_KWARGS.items()}
        if self.custom_path is not None:
            for k, v in _custom_rules(self.custom_path).items():
                out.setdefault(k, v)  # a built-in name wins, as in the rule loader (config_parser.py:213-233)
        return out

    def get_observations(self):
        return sorted(set(list(_spec._POS_TAGS) + ['Self', 'Other', 'Agent', 'Combined', 'Placeholder', 'Battery',
                                                   'GlobalPosition', 'Inventory', 'Destination', 'Defaults']))

    def get_all(self):
        out = dict(self.get_general_section())
        out.update(self.get_agent_section())
        out['Entities'] = self.get_entities()
        out['Rules'] = self.get_rules()
        return out

    @staticmethod
    def _save(data, path):
        path = Path(path)
        path.parent.mkdir(parents=True, exist_ok=True)
        with path.open('w') as f:
            yaml.safe_dump(data, f, sort_keys=False)
        return path

    def save_actions(self, output_conf_file='actions.yml'):
        return self._save(self.get_actions(), output_conf_file)

    def save_entities(self, output_conf_file='entities.yml'):
        return self._save(self.get_entities(), output_conf_file)

    def save_observations(self, output_conf_file='observations.yml'):
        return self._save(self.get_observations(), output_conf_file)

    def save_rules(self, output_conf_file='rules.yml'):
        return self._save(self.get_rules(), output_conf_file)

    def save_all(self, output_conf_file='all.yml'):
        return self._save(self.get_all(), output_conf_file)

"""`marl_factory_grid.environment.rules.Rule` for custom rule modules.

The built-in rules run inside the HIP engine; a user Rule subclass found in `custom_modules_path` runs on the
host (mfg_amd/host_rules.py) with the reference's hook API (environment/rules.py:14-142): every hook returns
a list of Results (or None) and receives a read-only view of the env state.
"""
import abc


class Rule(abc.ABC):

    @property
    def name(self):
        return self.__class__.__name__

    def __init__(self):
        pass

    def __repr__(self):
        return f'{self.name}'

    def on_init(self, state, lvl_map):
        return []

    def on_reset_post_spawn(self, state):
        return []

    def on_reset(self, state):
        return []

    def tick_pre_step(self, state):
        return []

    def tick_step(self, state):
        return []

    def tick_post_step(self, state):
        return []

    def on_check_done(self, state):
        return []

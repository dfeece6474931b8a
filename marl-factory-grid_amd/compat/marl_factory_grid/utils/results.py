"""Result records for custom rule modules (the reference's utils/results.py:23-104 field layout):
`identifier`, `validity`, `reward`, `value`, `collision`, `entity`. mfg_amd/host_rules.py folds them into
the step's rewards and info exactly like Factory.summarize_step_results."""
from dataclasses import dataclass
from typing import Any, Optional, Union

TYPE_VALUE, TYPE_REWARD = 'value', 'reward'


@dataclass
class InfoObject:
    identifier: str
    val_type: str
    value: Union[float, int]


@dataclass
class Result:
    identifier: str
    validity: bool
    reward: Optional[float] = None
    value: Optional[float] = None
    collision: Optional[bool] = None
    entity: Any = None

    def get_infos(self):
        n = self.entity.name if self.entity is not None else 'Global'
        return [InfoObject(f'{n}_{self.identifier}', t, getattr(self, t)) for t in (TYPE_VALUE, TYPE_REWARD)
                if getattr(self, t) is not None]


class ActionResult(Result):
    def __init__(self, *args, action_introduced_collision: bool = False, **kwargs):
        super().__init__(*args, **kwargs)
        self.action_introduced_collision = action_introduced_collision


@dataclass
class DoneResult(Result):
    pass


@dataclass
class TickResult(Result):
    pass


@dataclass
class State(Result):
    pass

"""Custom rules for the host-rule fallback tests. Written against the reference's plugin
API (environment/rules.py Rule hooks, utils/results.py TickResult/DoneResult); the same file is loaded by
the reference (tools/gen_golden_custom.py) and by mfg_amd.Factory(custom_modules_path=...)."""
from collections import Counter

from marl_factory_grid.environment.rules import Rule
from marl_factory_grid.utils.results import TickResult, DoneResult
import marl_factory_grid.environment.constants as c


class DoorProximityBonus(Rule):
    """tick_post_step: `bonus` for every agent on or next to a door."""

    def __init__(self, bonus=0.05):
        super().__init__()
        self.bonus = bonus

    def tick_post_step(self, state):
        doors = [d.pos for d in state['Doors']]
        res = []
        for agent in state[c.AGENT]:
            x, y = agent.pos
            if any(abs(x - dx) <= 1 and abs(y - dy) <= 1 for dx, dy in doors):
                res.append(TickResult(self.name, validity=c.VALID, reward=self.bonus, entity=agent))
        return res


class CountFailedActions(Rule):
    """tick_step: a global value result, the number of agents whose action failed this step."""

    def tick_step(self, state):
        n = sum(1 for a in state[c.AGENT] if not a.state.validity)
        return [TickResult(self.name, validity=c.VALID, value=n)]


class PenaltyBeforeActions(Rule):
    """tick_pre_step: a small global penalty every 7th step (curr_step is already advanced)."""

    def tick_pre_step(self, state):
        if state.curr_step % 7 == 0:
            return [TickResult(self.name, validity=c.VALID, reward=-0.125)]
        return []


class DoneWhenCrowded(Rule):
    """on_check_done: done with `reward` when at least `k` agents share one cell."""

    def __init__(self, k=3, reward=-1.0):
        super().__init__()
        self.k, self.reward = k, reward

    def on_check_done(self, state):
        cnt = Counter(tuple(a.pos) for a in state[c.AGENT])
        if cnt and max(cnt.values()) >= self.k:
            return [DoneResult(self.name, validity=c.VALID, reward=self.reward)]
        return [DoneResult(self.name, validity=c.NOT_VALID)]

"""Reference-compatible host layer over the HIP engine.

`Factory` mirrors `marl_factory_grid.environment.factory.Factory` (environment/factory.py:21-292) for ONE
env: same constructor arguments, `reset() -> {agent name: ndarray (L, d, d) float64}`,
`step(actions) -> (None, [ndarray per agent], reward, done, info)` with the identical info dict (rebuilt
from the engine's event record, mfg_amd/info.py), `action_space` / `named_action_space` /
`observation_space` / `named_observation_space`, and the same error behaviour for unsupported configs
(a clean `UnsupportedSpec`). The reference draws every shuffle from Python's global `random`; the
facade imports that MT19937 state into the engine before each call and writes the advanced state back
after it (`sync_python_random=True`), so `random.seed(s); env = Factory(cfg)` reproduces the
reference's trajectories AND leaves `random` where the reference would.

`BatchedFactory` is the training-loop interface: B envs on one GPU, torch tensors in and out
(obs [B, A, Lmax, d, d], reward [B, A] f64, done [B] u8, event rows for the info columns), auto-reset
with reference reset semantics. There is no CPU fallback: both raise without the HIP library or a GPU.
"""
import random as _pyrandom

import numpy as np

from . import abi
from .engine import Engine, PackedObs, RecordView, events_from_rows, EV_MISC, HDR, HDR_N
from .host_rules import HostRules, StaleStateError, StateView, fold_step, level_map, pre_snapshot
from .info import rebuild_info
from .spec import compile_spec, UnsupportedSpec
from . import views as _views

INIT_CREATE, INIT_KEEP_MT, INIT_NO_RESET = 1, 2, 4  # include/mfg.h MFG_INIT_*


class _Discrete:
    """Minimal stand-in for gymnasium.spaces.Discrete when gymnasium is not installed."""

    def __init__(self, n):
        self.n = int(n)

    def __repr__(self):
        return f'Discrete({self.n})'

    def __eq__(self, o):
        return getattr(o, 'n', None) == self.n


class _Tuple(tuple):
    def __repr__(self):
        return f'Tuple({", ".join(map(repr, self))})'


class _Box:
    def __init__(self, low, high, shape, dtype):
        self.low, self.high, self.shape, self.dtype = low, high, tuple(shape), dtype

    def __repr__(self):
        return f'Box({self.low}, {self.high}, {self.shape}, {np.dtype(self.dtype).name})'


def _spaces():
    try:
        from gymnasium import spaces
        return spaces.Discrete, spaces.Tuple, spaces.Box
    except ImportError:
        return _Discrete, (lambda xs: _Tuple(xs)), _Box


class Factory:
    """One env of the factory grid-world on the MI355X engine, reference API (factory.py:81)."""

    def __init__(self, config_file, custom_modules_path=None, custom_level_path=None, *, device=0,
                 sync_python_random=True, py_seed=None):
        import torch
        self._torch = torch
        self._config_file = config_file
        # custom Rule classes from custom_modules_path run on the host beside the engine (mfg_amd/host_rules.py)
        self.spec = compile_spec(config_file, custom_level_path, custom_modules_path)
        self._host = HostRules(self.spec) if self.spec.host_rules else None
        self._host_init = False
        self._eng = Engine(self.spec, 1, device=device)
        self._dev = self._eng.device
        self._sync = sync_python_random and py_seed is None
        A, s = self.spec.n_agents, self.spec
        self._obs = torch.zeros(self._eng.obs_shape(), dtype=torch.float64, device=self._dev)
        self._rew = torch.zeros((1, A), dtype=torch.float64, device=self._dev)
        self._done = torch.zeros(1, dtype=torch.uint8, device=self._dev)
        self._ev_a = torch.zeros((1, A), dtype=torch.uint8, device=self._dev)
        self._ev_w = torch.zeros((1, A), dtype=torch.uint8, device=self._dev)
        self._ev_m = torch.zeros((1, EV_MISC), dtype=torch.int32, device=self._dev)
        self._act = torch.zeros((1, A), dtype=torch.int32, device=self._dev)
        self._step = 0
        self._agent_states = None  # agent.state per agent after the last step (None: all Noop/valid)
        self._manual = None        # manual_* protocol: actions collected since manual_step_init
        self._last = None          # (reward, done, info) of the last executed step
        self._stale_step = False   # a host rule's StaleStateError ended the last step: reset() before stepping
        # Factory.__init__: entities, rules, OBSBuilder (its floor-list access shuffles once, Q3)
        if self._sync:
            self._push_random()
            self._eng.reset(obs=None, init=INIT_CREATE | INIT_KEEP_MT | INIT_NO_RESET)
            self._pull_random()
        else:
            self._eng.reset(obs=None, init=INIT_CREATE | INIT_NO_RESET, seed_base=int(py_seed or 0))

    # ---- Python `random` <-> engine MT19937 ----
    def _push_random(self):
        st = self._eng.export_state()
        rec = st[0].cpu().numpy().copy()
        L = self._eng.layout
        ver, internal, _ = _pyrandom.getstate()
        words = np.asarray(internal[:624], dtype=np.uint32)
        rec[L['o_mt']:L['o_mt'] + 4 * 624] = words.view(np.uint8)
        hdr = rec[L['o_hdr']:L['o_hdr'] + 4 * HDR_N].view(np.int32)
        hdr[HDR['mt_idx']] = int(internal[624])
        self._eng.import_state(self._torch.from_numpy(rec).to(self._dev).reshape(1, -1))

    def _pull_random(self):
        mt = self._view().mt()
        _pyrandom.setstate((3, tuple(int(x) for x in mt[:624]) + (int(mt[624]),), None))

    def _view(self):
        return RecordView(self._eng.export_state()[0].cpu().numpy(), self._eng.layout, self.spec)

    # ---- reference API ----
    @property
    def action_space(self):
        Discrete, Tuple, _ = _spaces()
        return Tuple([Discrete(n) for n in self.spec.n_actions])

    @property
    def named_action_space(self):
        return {f'Agent[{n}]': {a: i for i, a in enumerate(self.spec.action_idents[k])}
                for k, n in enumerate(self.spec.agent_names)}

    @property
    def observation_space(self):
        _, Tuple, Box = _spaces()
        hw, nl = tuple(self.spec.obs_hw), self.spec.n_layers
        boxes = [Box(low=0, high=1, shape=(nl[a],) + hw, dtype=np.float32) for a in range(self.spec.n_agents)]
        return boxes[0] if len(boxes) == 1 else Tuple(boxes)

    @property
    def named_observation_space(self):
        return {f'Agent[{n}]': list(self.spec.layer_names[k]) for k, n in enumerate(self.spec.agent_names)}

    @property
    def params(self):
        import yaml
        with open(self.spec.config_path) as f:
            return yaml.safe_load(f)

    def _obs_list(self):
        o = self._obs[0].cpu().numpy()
        return [o[a, :self.spec.n_layers[a]].copy() for a in range(self.spec.n_agents)]

    def reset(self):
        """factory.py:134-148: reset state and entities, spawn, return the first observation per agent."""
        if self._sync:
            self._push_random()
        self._eng.reset(obs=self._obs, init=0)
        if self._sync:
            self._pull_random()
        self._torch.cuda.synchronize(self._dev)
        self._agent_states = None
        self._step = 0
        self._stale_step = False
        if self._host:
            view = StateView(self.spec, self.snapshot())
            if not self._host_init:  # rules.do_all_init (factory.py:121); the view is the reset state here
                self._host.on_init(view, level_map(self.spec))
                self._host_init = True
            self._host.on_reset(view)
        return {f'Agent[{n}]': o for n, o in zip(self.spec.agent_names, self._obs_list())}

    def step(self, actions):
        """factory.py:189-220. Returns (None, obs list, reward, done, info)."""
        if self._stale_step:
            raise RuntimeError('a custom rule raised StaleStateError in the last step after the engine had already '
                               'executed it; call reset() before stepping again')
        if not isinstance(actions, list):
            actions = [int(actions)]
        A = self.spec.n_agents
        if len(actions) != A:
            raise ValueError(f'expected {A} actions, got {len(actions)}')
        for a, x in enumerate(actions):
            if not 0 <= int(x) < self.spec.n_actions[a]:
                raise IndexError(f'action {x} out of range for agent {a}')
        self._act.copy_(self._torch.tensor([actions], dtype=self._torch.int32))
        pre = None
        if self._host:  # the state the host rules' tick_pre_step sees: before the actions (states.py:181-187)
            pre = pre_snapshot(self.snapshot())
        if self._sync:
            self._push_random()
        self._eng.step(1, actions=self._act, reward=self._rew, done=self._done, obs=self._obs, ev_act=self._ev_a,
                       ev_watch=self._ev_w, ev_misc=self._ev_m, auto_reset=False)
        if self._sync:
            self._pull_random()
        ev_a, ev_w = self._ev_a[0].cpu().numpy(), self._ev_w[0].cpu().numpy()
        ev = events_from_rows(ev_a, ev_w, self._ev_m[0].cpu().numpy())
        if ev['crashed']:
            raise RuntimeError('the reference crashes on this step (SURVEY App. A Q9/Q17); env state is flagged')
        reward = [float(x) for x in self._rew[0].cpu().numpy()]
        done = bool(self._done.item())
        self._step = ev['step']
        self._agent_states = _views.agent_states(self.spec, actions, ev_a, ev_w)
        if self._host:  # custom rules: their Results join the device's in rule order, then one fold
            try:
                reward, done, info = fold_step(self.spec, self._host, [int(x) for x in actions], ev, pre,
                                               self.snapshot(), done)
            except BaseException:  # StaleStateError or anything custom rule code raises inside the fold
                self._stale_step = True  # the device stepped but this step's results were never returned
                raise
            info = dict(info)
        else:
            info = dict(rebuild_info(self.spec, [int(x) for x in actions], ev, reward))
        self._last = (reward, done, info)
        return None, self._obs_list(), reward, done, info

    # ---- entity views (factory.py:131-132, 262-292) ----
    def snapshot(self):
        """The env's state as a `views.Snapshot` (one device->host copy of the record)."""
        return _views.snapshot_from_record(self._view(), self._agent_states)

    def __getitem__(self, item):
        """`env['Doors']` etc.: a read-only `views.GroupView` of the collection (factory.py:131-132)."""
        return _views.group_view(self.spec, self.snapshot(), item)

    def summarize_state(self):
        return _views.summarize_state(self.spec, self.snapshot())

    def summarize_header(self):
        return _views.summarize_header(self.spec, self.snapshot())

    def render(self, mode='human'):
        """factory.py:262-273. The reference draws `state.entities.render()` with pygame; here 'human' prints
        a text frame, 'ansi' returns it, 'entities' returns the RenderEntity list and 'rgb_array' an
        (H, W, 3) uint8 image of it."""
        snap = self.snapshot()
        if mode == 'entities':
            return _views.render_entities(self.spec, snap)
        if mode == 'rgb_array':
            return _views.render_rgb(self.spec, snap)
        frame = _views.render_ansi(self.spec, snap)
        if mode == 'ansi':
            return frame
        print(frame)
        return None

    def save_params(self, filepath):
        """factory.py:294-298: copy the config file."""
        import shutil
        from pathlib import Path
        filepath = Path(filepath)
        filepath.parent.mkdir(parents=True, exist_ok=True)
        shutil.copyfile(self.spec.config_path, filepath)

    # ---- manual stepping (factory.py:150-187) ----
    # The engine runs a whole step (pre-step rules, every agent in list order, step/post-step rules) in one
    # device pass, so the manual protocol collects the agents' actions and executes the step at
    # manual_finalize_init. Agents must be ticked once each, in list order; an agent's ActionResult is
    # available after manual_finalize_init (ManualResult.resolve).
    def manual_step_init(self):
        self._manual = []
        return []

    def manual_agent_tick(self, agent_name, action):
        if self._manual is None:
            raise RuntimeError('manual_agent_tick before manual_step_init')
        names = [f'Agent[{n}]' for n in self.spec.agent_names]
        key = agent_name if agent_name in names else f'Agent[{agent_name}]'
        if key not in names:
            raise KeyError(f'"{agent_name}" could not be found. Check the spelling!')
        a = names.index(key)
        if a != len(self._manual):
            raise RuntimeError('the engine executes agents in list order: tick each agent once, in order '
                               f'(expected {names[len(self._manual)]}, got {key})')
        if not 0 <= int(action) < self.spec.n_actions[a]:
            raise IndexError(f'action {action} out of range for {key}')
        self._manual.append(int(action))
        return ManualResult(self, a)

    def manual_finalize_init(self):
        if self._manual is None or len(self._manual) != self.spec.n_agents:
            raise RuntimeError('manual_finalize_init needs one manual_agent_tick per agent')
        acts, self._manual = self._manual, None
        self.step(acts)
        return []

    def manual_step_finalize(self, tick_result=None):
        if self._last is None:
            raise RuntimeError('no step has been executed')
        return self._last

    def manual_get_named_agent_obs(self, agent_name):
        names = [f'Agent[{n}]' for n in self.spec.agent_names]
        key = agent_name if agent_name in names else f'Agent[{agent_name}]'
        a = names.index(key)
        return list(self.spec.layer_names[a]), self._obs_list()[a]

    def manual_get_agent_obs(self, agent_name):
        return self.manual_get_named_agent_obs(agent_name)[1]

    def close(self):
        if getattr(self, '_eng', None) is not None:
            self._eng.close()
            self._eng = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


class ManualResult:
    """An agent's action result in the manual protocol, filled in once the step has executed."""

    def __init__(self, env, agent):
        self._env, self._a = env, agent

    def resolve(self):
        st = self._env._agent_states
        if st is None:
            raise RuntimeError('the step has not been executed yet (call manual_finalize_init)')
        return st[self._a]

    @property
    def identifier(self):
        return self.resolve()[0]

    @property
    def validity(self):
        return self.resolve()[1]


class BatchedFactory:
    """B envs of one config on one GPU: torch tensors in and out, auto-reset."""

    def __init__(self, config_file, n_envs, *, device=0, seed_base=0, obs_dtype='float32', custom_level_path=None,
                 packed_cap=32, proj_weight=None, proj_bias=None):
        """obs_dtype 'float32' / 'float64': dense obs [B, A, lmax, h, w]; 'packed': an engine.PackedObs
        (nonzero entries per agent row, cap `packed_cap`, plus the fused projection when `proj_weight`, an
        nn.Linear(lmax*h*w, E).weight, is given)."""
        import torch
        self.torch = torch
        self.spec = compile_spec(config_file, custom_level_path)
        self.B = int(n_envs)
        self.engine = Engine(self.spec, self.B, device=device)
        self.device = self.engine.device
        self.seed_base = int(seed_base)
        A = self.spec.n_agents
        if obs_dtype == 'packed':
            self.obs = PackedObs(self.engine, K=1, cap=packed_cap, weight=proj_weight, bias=proj_bias)
        else:
            dt = {'float32': torch.float32, 'float64': torch.float64}[obs_dtype]
            self.obs = torch.zeros(self.engine.obs_shape(), dtype=dt, device=self.device)
        self.reward = torch.zeros((self.B, A), dtype=torch.float64, device=self.device)
        self.done = torch.zeros(self.B, dtype=torch.uint8, device=self.device)
        self.ev_act = torch.zeros((self.B, A), dtype=torch.uint8, device=self.device)
        self.ev_watch = torch.zeros((self.B, A), dtype=torch.uint8, device=self.device)
        self.ev_misc = torch.zeros((self.B, EV_MISC), dtype=torch.int32, device=self.device)
        self._created = False
        self.t = 0

    @property
    def n_agents(self):
        return self.spec.n_agents

    def reset(self, mask=None):
        """Create (first call: env b seeded like random.seed(seed_base + b)) or reset envs; returns obs."""
        init = 0 if self._created else INIT_CREATE
        self.engine.reset(obs=self.obs, mask=mask, init=init, seed_base=self.seed_base)
        self._created = True
        return self.obs

    def step(self, actions):
        """actions: int32 tensor [B, A] on the device. Returns (obs, reward, done, events)."""
        if not self._created:
            raise RuntimeError('call reset() first')
        a = actions.to(device=self.device, dtype=self.torch.int32).contiguous()
        if a.shape != (self.B, self.spec.n_agents):
            raise ValueError(f'actions must be [{self.B}, {self.spec.n_agents}]')
        self.engine.step(1, actions=a, reward=self.reward, done=self.done, obs=self.obs, ev_act=self.ev_act,
                         ev_watch=self.ev_watch, ev_misc=self.ev_misc, auto_reset=True, step_base=self.t)
        self.t += 1
        return self.obs, self.reward, self.done, (self.ev_act, self.ev_watch, self.ev_misc)

    def rollout(self, K, philox_seed, obs=None, reward=None, done=None):
        """K steps with on-device Philox synthetic actions into caller buffers [K, ...] (any may be None)."""
        self.engine.step(K, actions=None, philox_seed=philox_seed, env_base=self.seed_base, step_base=self.t,
                         reward=reward, done=done, obs=obs, auto_reset=True)
        self.t += K

    def info(self, b, actions):
        """The reference info dict of env b's last step (host-side rebuild from the event rows)."""
        ev = events_from_rows(self.ev_act[b].cpu().numpy(), self.ev_watch[b].cpu().numpy(),
                              self.ev_misc[b].cpu().numpy())
        return dict(rebuild_info(self.spec, [int(x) for x in actions], ev,
                                 [float(x) for x in self.reward[b].cpu().numpy()]))

    def info_columns(self, actions):
        """The last step's info dicts of all B envs as device columns (mfg_amd.info_columns): returns
        (names, values f64 [B, K], present bool [B, K]); no host copy."""
        if getattr(self, '_info_cols', None) is None:
            from .info_columns import InfoColumns
            self._info_cols = InfoColumns(self.spec)
        v, p = self._info_cols(actions, self.ev_act, self.ev_watch, self.ev_misc, self.reward)
        return self._info_cols.columns, v, p

    def close(self):
        self.engine.close()

"""Vector-env and multi-agent adapters over the engine.

Training code written against the usual env interfaces drops in without touching the engine:

* `VectorFactory` -- gymnasium.vector-style batch interface over `BatchedFactory`: `reset(seed, options)
  -> (obs, infos)`, `step(actions) -> (obs, rewards, terminations, truncations, infos)`, torch tensors
  on the device (obs [B, A, L, d, d], rewards [B, A] f64). Auto-reset happens inside the step (the obs
  of a finished env is its next episode's first obs); per-episode returns and lengths are kept on the
  device and reported for the envs that finished.
* `ParallelFactory` -- PettingZoo ParallelEnv-style dict interface over the B=1 `Factory` facade.
* `SB3VecFactory` -- stable-baselines3 VecEnv-style numpy interface (joint action MultiDiscrete, the
  agents' rewards summed), over `VectorFactory`.

The reference has one done flag (factory.py:216-220). Here a done whose only cause is
DoneAtMaxStepsReached (rules.py:202-225) is a truncation, every other done a termination. gymnasium,
pettingzoo and stable-baselines3 are not installed in this image; the spaces come from gymnasium when it
is importable, else from the minimal stand-ins of `mfg_amd.factory`.
"""
import numpy as np

from . import abi
from .factory import BatchedFactory, Factory, _spaces


def _maxsteps_bits(spec):
    """done_mask bits of the DoneAtMaxStepsReached rules, and of all done rules."""
    ms = 0
    for ri, (op, _, _) in enumerate(spec.rules):
        if op == abi.RULE_DONE_MAXSTEPS:
            ms |= 1 << ri
    return ms


class VectorFactory:
    """B envs of one config on one GPU with a gymnasium.vector-like interface."""

    metadata = {'autoreset_mode': 'same-step'}

    def __init__(self, config_file, num_envs, *, device=0, seed_base=0, obs_dtype='float32', env=None):
        self.env = env if env is not None else BatchedFactory(config_file, num_envs, device=device,
                                                                seed_base=seed_base, obs_dtype=obs_dtype)
        self.torch = self.env.torch
        self.spec = self.env.spec
        self.num_envs = self.env.B
        self.n_agents = self.spec.n_agents
        self.agent_names = [f'Agent[{n}]' for n in self.spec.agent_names]
        self._ms_bits = _maxsteps_bits(self.spec)
        dev = self.env.device
        self._ret = self.torch.zeros((self.num_envs, self.n_agents), dtype=self.torch.float64, device=dev)
        self._len = self.torch.zeros(self.num_envs, dtype=self.torch.int64, device=dev)
        Discrete, Tuple, Box = _spaces()
        hw, nl = tuple(self.spec.obs_hw), self.spec.n_layers
        self.single_action_space = Tuple([Discrete(n) for n in self.spec.n_actions])
        self.single_observation_space = Tuple([Box(0, 1, (nl[a],) + hw, np.float32) for a in range(self.n_agents)])

    def reset(self, seed=None, options=None):
        """Create (first call) or reset every env (options={'mask': bool tensor [B]} resets a subset). A
        `seed` re-seeds the envs: env b as `random.seed(seed + b)` would in the reference."""
        mask = (options or {}).get('mask')
        if seed is not None:
            self.env.seed_base = int(seed)
            self.env._created = False
        m = None if mask is None else mask.to(device=self.env.device, dtype=self.torch.uint8)
        obs = self.env.reset(mask=m)
        if m is None:
            self._ret.zero_()
            self._len.zero_()
        else:
            keep = (m == 0)
            self._ret.mul_(keep.unsqueeze(1).to(self._ret.dtype))
            self._len.mul_(keep.to(self._len.dtype))
        return obs, {}

    def step(self, actions):
        obs, rew, done, (_, _, ev_misc) = self.env.step(actions)
        done_b = done.bool()
        dm = ev_misc[:, 7].to(self.torch.int64) & 0xFFFFFFFF
        trunc = done_b & ((dm & ~self._ms_bits) == 0) & ((dm & self._ms_bits) != 0)
        term = done_b & ~trunc
        self._ret += rew
        self._len += 1
        # every step carries the final-episode columns (zero where not done): no device->host sync per step
        infos = {'done_mask': dm,
                 'final_return': self.torch.where(done_b.unsqueeze(1), self._ret, self.torch.zeros_like(self._ret)),
                 'final_length': self.torch.where(done_b, self._len, self.torch.zeros_like(self._len)),
                 '_final': done_b.clone()}
        self._ret.masked_fill_(done_b.unsqueeze(1), 0.0)
        self._len.masked_fill_(done_b, 0)
        return obs, rew, term, trunc, infos

    def close(self):
        self.env.close()


class ParallelFactory:
    """One env with a PettingZoo ParallelEnv-like interface (dicts keyed by agent name)."""

    metadata = {'render_modes': ['human', 'ansi', 'rgb_array'], 'name': 'marl_factory_grid_amd'}

    def __init__(self, config_file, *, device=0, py_seed=0, render_mode=None):
        self._cfg, self._device, self._seed = config_file, device, int(py_seed)
        self.render_mode = render_mode
        self.env = Factory(config_file, device=device, py_seed=self._seed)
        self.spec = self.env.spec
        self.possible_agents = [f'Agent[{n}]' for n in self.spec.agent_names]
        self.agents = []
        self._ms_bits = _maxsteps_bits(self.spec)

    def observation_space(self, agent):
        _, _, Box = _spaces()
        a = self.possible_agents.index(agent)
        return Box(0, 1, (self.spec.n_layers[a],) + tuple(self.spec.obs_hw), np.float32)

    def action_space(self, agent):
        Discrete, _, _ = _spaces()
        return Discrete(self.spec.n_actions[self.possible_agents.index(agent)])

    def reset(self, seed=None, options=None):
        if seed is not None and int(seed) != self._seed:  # as random.seed(seed); Factory(cfg) would
            self.env.close()
            self._seed = int(seed)
            self.env = Factory(self._cfg, device=self._device, py_seed=self._seed)
        obs = self.env.reset()
        self.agents = list(self.possible_agents)
        return dict(obs), {a: {} for a in self.agents}

    def step(self, actions):
        acts = [int(actions[a]) for a in self.possible_agents]
        _, obs, rew, done, info = self.env.step(acts)
        dm = int(self.env._ev_m[0, 7].item()) & 0xFFFFFFFF
        trunc = done and (dm & ~self._ms_bits) == 0 and (dm & self._ms_bits) != 0
        names = self.possible_agents
        out = ({a: o for a, o in zip(names, obs)}, {a: r for a, r in zip(names, rew)},
               {a: bool(done and not trunc) for a in names}, {a: bool(trunc) for a in names},
               {a: dict(info) for a in names})
        if done:
            self.agents = []
        return out

    def render(self):
        return self.env.render(self.render_mode or 'ansi')

    def state(self):
        return self.env.summarize_state()

    def close(self):
        self.env.close()


class SB3VecFactory:
    """stable-baselines3 VecEnv-like numpy interface over `VectorFactory`: obs [B, A*L, d, d] float32, the
    joint action [B, A] (MultiDiscrete of the agents' action counts), reward = the agents' sum."""

    def __init__(self, config_file, num_envs, *, device=0, seed_base=0, venv=None):
        self.venv = venv if venv is not None else VectorFactory(config_file, num_envs, device=device,
                                                                 seed_base=seed_base)
        self.num_envs = self.venv.num_envs
        spec = self.venv.spec
        self._L = max(spec.n_layers)
        _, _, Box = _spaces()
        self.observation_space = Box(0, 1, (spec.n_agents * self._L,) + tuple(spec.obs_hw), np.float32)
        self.action_space = _multidiscrete(spec.n_actions)
        self._actions = None

    def _np_obs(self, obs):
        o = obs.float().reshape(self.num_envs, -1, obs.shape[-2], obs.shape[-1])
        return o.cpu().numpy()

    def reset(self):
        obs, _ = self.venv.reset()
        return self._np_obs(obs)

    def step_async(self, actions):
        self._actions = np.asarray(actions, dtype=np.int32).reshape(self.num_envs, -1)

    def step_wait(self):
        a = self.venv.torch.from_numpy(self._actions).to(self.venv.env.device)
        obs, rew, term, trunc, infos = self.venv.step(a)
        dones = (term | trunc).cpu().numpy()
        r = rew.sum(dim=1).cpu().numpy().astype(np.float32)
        tr = trunc.cpu().numpy()
        info_list = [{'TimeLimit.truncated': bool(tr[b])} for b in range(self.num_envs)]
        if '_final' in infos:
            fr = infos['final_return'].sum(dim=1).cpu().numpy()
            fl = infos['final_length'].cpu().numpy()
            for b in np.nonzero(dones)[0]:
                info_list[b]['episode'] = {'r': float(fr[b]), 'l': int(fl[b])}
        return self._np_obs(obs), r, dones, info_list

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def close(self):
        self.venv.close()

    def get_attr(self, name, indices=None):
        return [getattr(self.venv, name)] * (self.num_envs if indices is None else len(list(indices)))

    def set_attr(self, name, value, indices=None):
        setattr(self.venv, name, value)

    def env_method(self, name, *args, indices=None, **kwargs):
        r = getattr(self.venv, name)(*args, **kwargs)
        return [r] * (self.num_envs if indices is None else len(list(indices)))

    def env_is_wrapped(self, wrapper_class, indices=None):
        return [False] * (self.num_envs if indices is None else len(list(indices)))

    def seed(self, seed=None):
        if seed is not None:
            self.venv.reset(seed=seed)
        return [None if seed is None else seed + b for b in range(self.num_envs)]


class _MultiDiscrete:
    """Minimal stand-in for gymnasium.spaces.MultiDiscrete."""

    def __init__(self, nvec):
        self.nvec = np.asarray(nvec, np.int64)
        self.shape = self.nvec.shape

    def __repr__(self):
        return f'MultiDiscrete({self.nvec.tolist()})'


def _multidiscrete(nvec):
    try:
        from gymnasium.spaces import MultiDiscrete
        return MultiDiscrete(nvec)
    except ImportError:
        return _MultiDiscrete(nvec)

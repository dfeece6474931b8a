"""Vector-env / multi-agent adapters and the monitor/recorder wrappers.

CPU: the adapters' bookkeeping (termination vs truncation split of the reference's single done flag,
per-episode returns/lengths, SB3-style numpy views, EnvMonitor's per-episode aggregation,
EnvRecorder's record layout) over a scripted stand-in env with the engine's I/O contract.
GPU: the same adapters over the HIP engine."""
import json
import random

import numpy as np
import pytest
import torch

from conftest import gpu_available


class _ScriptedBatched:
    """Stand-in with BatchedFactory's I/O contract: env b finishes every (5 + b) steps; even envs by
    DoneAtMaxStepsReached (rule 1), odd ones by another done rule (rule 0); reward = b + 0.5 per agent."""

    def __init__(self, B=4, A=2):
        from mfg_amd import abi
        self.torch = torch
        self.B, self.device, self.seed_base, self._created = B, torch.device('cpu'), 0, False

        class S:
            n_agents, d = A, 3
            obs_hw = (3, 3)
            n_layers = [2] * A
            n_actions = [5] * A
            agent_names = [f'a{k}' for k in range(A)]
            rules = [(abi.RULE_DONE_DIRT, [], []), (abi.RULE_DONE_MAXSTEPS, [], [])]
        self.spec = S
        self.t = np.zeros(B, np.int64)

    def reset(self, mask=None):
        self._created = True
        if mask is None:
            self.t[:] = 0
        else:
            self.t[mask.cpu().numpy().astype(bool)] = 0
        return torch.zeros((self.B, self.spec.n_agents, 2, 3, 3))

    def step(self, actions):
        self.t += 1
        done = np.array([self.t[b] % (5 + b) == 0 for b in range(self.B)])
        dm = np.array([(2 if b % 2 == 0 else 1) if done[b] else 0 for b in range(self.B)], np.int32)
        ev_misc = torch.zeros((self.B, 12), dtype=torch.int32)
        ev_misc[:, 7] = torch.from_numpy(dm)
        rew = torch.tensor([[b + 0.5] * self.spec.n_agents for b in range(self.B)], dtype=torch.float64)
        self.t[done] = 0
        obs = torch.zeros((self.B, self.spec.n_agents, 2, 3, 3))
        return obs, rew, torch.from_numpy(done.astype(np.uint8)), (None, None, ev_misc)

    def close(self):
        pass


def test_vector_factory_bookkeeping():
    from mfg_amd.vec import VectorFactory
    from mfg_amd.monitor import BatchedEpisodeLog
    v = VectorFactory(None, None, env=_ScriptedBatched())
    v.reset()
    log = BatchedEpisodeLog()
    seen = 0
    for t in range(1, 31):
        obs, rew, term, trunc, infos = v.step(torch.zeros((4, 2), dtype=torch.int32))
        for b in range(4):
            done = t % (5 + b) == 0
            assert bool(term[b] | trunc[b]) == done
            if done:
                assert bool(trunc[b]) == (b % 2 == 0) and bool(term[b]) == (b % 2 == 1)
                assert infos['final_length'][b].item() == 5 + b
                assert infos['final_return'][b, 0].item() == (5 + b) * (b + 0.5)
        seen += log.update(infos)
    df = log.frame()
    assert len(df) == seen == sum(30 // (5 + b) for b in range(4))
    assert (df['return_sum'] == df['length'] * (df['env'] + 0.5) * 2).all()


def test_sb3_view():
    from mfg_amd.vec import SB3VecFactory, VectorFactory
    s = SB3VecFactory(None, None, venv=VectorFactory(None, None, env=_ScriptedBatched()))
    assert s.reset().shape == (4, 4, 3, 3)
    for t in range(1, 6):
        obs, r, dones, infos = s.step(np.zeros((4, 2), np.int32))
    assert dones[0] and not dones[1]
    assert infos[0]['TimeLimit.truncated'] and infos[0]['episode'] == {'r': 5.0, 'l': 5}
    assert r.dtype == np.float32 and r[1] == 3.0
    assert s.get_attr('num_envs') == [4] * 4 and s.env_is_wrapped(object) == [False] * 4


class _ScriptedFactory:
    params = {'General': {'level_name': 'x', 'pomdp_r': 3, 'env_seed': 69}, 'Agents': {'a': {}}}

    def __init__(self):
        self.t = 0

    def reset(self):
        self.t = 0
        return {}

    def step(self, actions):
        self.t += 1
        info = {'Agent[a]_North': -0.001, 'Global_DoorAutoClose': 1.0, 'step_reward': -0.001, 'step': self.t,
                'Agent[a]_Collisions_count': float(self.t)}
        return None, [], [-0.001], self.t % 4 == 0, info

    def summarize_state(self):
        return {'step': self.t, 'agents': [{'name': 'Agent[a]', 'x': self.t, 'y': 0}]}

    def summarize_header(self):
        return {'rec_step': self.t}


def test_env_monitor_aggregation(tmp_path):
    import pandas as pd
    from mfg_amd.monitor import EnvMonitor
    m = EnvMonitor(_ScriptedFactory(), tmp_path / 'mon.pick')
    m.reset()
    for _ in range(8):
        m.step([0])
    df = m.monitor_df
    assert len(df) == 2 and list(df['episode']) == [0, 1]
    assert df['Agent[a]_North'][0] == pytest.approx(-0.004) and df['Global_DoorAutoClose'][1] == 4.0
    assert df['Agent[a]_Collisions_count'][0] == 2.5 and df['Agent[a]_Collisions_count'][1] == 6.5  # '...ount': mean
    assert 'step' not in df.columns
    m.save_monitor()
    back = pd.read_pickle(tmp_path / 'mon.pick')  # our own file
    assert len(back) == 2


def test_env_recorder_layout(tmp_path):
    from mfg_amd.monitor import EnvRecorder
    r = EnvRecorder(_ScriptedFactory(), tmp_path / 'rec.json', episodes=[1])
    r.reset()
    for _ in range(6):
        r.step([0])
    out = json.loads(r.save_records().read_text())
    assert out['n_episodes'] == 1 and out['header'] == {'rec_step': 6}
    assert [len(e['steps']) for e in out['episodes']] == [4, 2]
    assert out['episodes'][0]['steps'][0]['agents'][0]['x'] == 1
    assert out['metadata']['level_name'] == 'x'


@pytest.mark.gpu
def test_vector_factory_on_engine():
    if not gpu_available():
        pytest.skip('no GPU')
    from mfg_amd.vec import VectorFactory
    from mfg_amd.monitor import BatchedEpisodeLog
    B = 64
    v = VectorFactory('rooms4.yaml', B, seed_base=5)
    obs, _ = v.reset()
    assert obs.shape[:2] == (B, v.n_agents)
    g = torch.Generator().manual_seed(0)
    ret = torch.zeros((B, v.n_agents), dtype=torch.float64)
    log = BatchedEpisodeLog()
    n_done = 0
    for t in range(520):
        a = torch.stack([torch.randint(0, n, (B,), generator=g) for n in v.spec.n_actions], 1).to(torch.int32)
        obs, rew, term, trunc, infos = v.step(a.to(v.env.device))
        ret += rew.cpu()
        d = (term | trunc).cpu()
        if d.any():
            assert torch.equal(infos['final_return'].cpu()[d], ret[d])
            ret[d] = 0
            n_done += int(d.sum())
        log.update(infos)
    assert n_done > 0 and len(log.frame()) == n_done
    v.close()


@pytest.mark.gpu
def test_parallel_factory_matches_facade():
    if not gpu_available():
        pytest.skip('no GPU')
    from mfg_amd.factory import Factory
    from mfg_amd.vec import ParallelFactory
    p = ParallelFactory('large8.yaml', py_seed=4)
    f = Factory('large8.yaml', py_seed=4)
    obs, infos = p.reset()
    ref = f.reset()
    assert list(obs) == p.possible_agents and all((obs[k] == ref[k]).all() for k in obs)
    rng = random.Random(1)
    for _ in range(30):
        acts = {a: rng.randrange(p.action_space(a).n) for a in p.agents}
        o, r, term, trunc, inf = p.step(acts)
        _, o2, r2, d2, i2 = f.step([acts[a] for a in p.possible_agents])
        assert [r[a] for a in p.possible_agents] == r2 and all((o[a] == x).all() for a, x in zip(p.possible_agents, o2))
        assert inf[p.possible_agents[0]] == i2
    p.close()
    f.close()


@pytest.mark.gpu
def test_monitor_and_recorder_on_engine(tmp_path):
    if not gpu_available():
        pytest.skip('no GPU')
    from mfg_amd.factory import Factory
    from mfg_amd.monitor import EnvMonitor, EnvRecorder
    env = EnvRecorder(EnvMonitor(Factory('rooms4.yaml', py_seed=2)), tmp_path / 'r.json')
    env.reset()
    rng = random.Random(0)
    for _ in range(510):
        _, _, _, done, _ = env.step([rng.randrange(n) for n in env.spec.n_actions])
        if done:
            env.reset()
    assert len(env.env.monitor_df) >= 1
    out = json.loads(env.save_records().read_text())
    assert out['episodes'][0]['steps'][0]['step'] == 1


def test_env_recorder_deltas_and_occupation(tmp_path):
    import numpy as np
    from mfg_amd.monitor import EnvRecorder, _deltas
    f = _ScriptedFactory()
    f.spec = type('S', (), {'H': 12, 'W': 3})()
    r = EnvRecorder(f, tmp_path / 'rec.json')
    r.reset()
    for _ in range(8):
        r.step([0])
    out = json.loads(r.save_records(only_deltas=True, save_occupation_map=True).read_text())
    assert len(out['episodes']) == 1  # one delta between the two recorded episodes
    d = out['episodes'][0]
    assert d['values_changed']["root['steps'][0]['step']"] == {'old_value': 1, 'new_value': 5}
    occ = np.load(tmp_path / 'rec_occupation.npy')
    assert occ.shape == (12, 3) and occ.sum() == 8 and occ[1:9, 0].tolist() == [1] * 8
    assert _deltas({'a': [1, 2]}, {'a': [1], 'b': 0}) == {'iterable_item_removed': {"root['a'][1]": 2},
                                                        'dictionary_item_added': {"root['b']": 0}}
    with pytest.raises(NotImplementedError):
        r.save_records(save_trajectory_map=True)


def test_env_monitor_auto_plot(tmp_path):
    from mfg_amd.monitor import EnvMonitor
    m = EnvMonitor(_ScriptedFactory(), tmp_path / 'mon.pick')
    m.reset()
    for _ in range(8):
        m.step([0])
    m.save_monitor(auto_plotting_keys=['Agent[a]_North'])
    assert (tmp_path / 'mon.png').exists() or (tmp_path / 'mon.csv').exists()

"""Host layer: the reference-compatible Factory facade and BatchedFactory.

CPU (always): the compat import path resolves to our facade, unsupported constructor arguments fail
cleanly, and without a GPU the facade raises instead of falling back to a CPU path.
GPU: `random.seed(s); env = Factory(cfg)` replays the reference fixtures exactly — rewards, done,
info dict, obs and the global `random` state after every call (the facade keeps Python's MT19937 in
step with the engine)."""
import random
import sys
from pathlib import Path

import numpy as np
import pytest

from conftest import gpu_available
import golden_compare as G

ROOT = Path(__file__).resolve().parent.parent
COMPAT = ROOT / 'marl-factory-grid_amd' / 'compat'


def test_compat_import_path():
    sys.path.insert(0, str(COMPAT))
    try:
        from marl_factory_grid.environment.factory import Factory
        from mfg_amd.factory import Factory as F2
        assert Factory is F2
    finally:
        sys.path.remove(str(COMPAT))


def test_custom_rule_missing_from_custom_path_rejected():
    """A rule found neither built in nor under custom_modules_path is a clean UnsupportedSpec (the reference
    exits, config_parser.py:238-249); found ones run on the host (tests/test_host_rules.py)."""
    from mfg_amd.factory import Factory
    from mfg_amd.spec import UnsupportedSpec
    with pytest.raises(UnsupportedSpec):
        Factory('custom_rules4.yaml', custom_modules_path='/tmp/nowhere')


def test_no_cpu_fallback():
    if gpu_available():
        pytest.skip('GPU present')
    from mfg_amd.factory import Factory, BatchedFactory
    with pytest.raises(RuntimeError):
        Factory('simple1.yaml')
    with pytest.raises(RuntimeError):
        BatchedFactory('simple1.yaml', 4)


@pytest.mark.gpu
@pytest.mark.parametrize('tag,cfg', [('large8', 'large8.yaml'), ('rooms4', 'rooms4.yaml'), ('simple1', 'simple1.yaml'),
                                     ('eight_puzzle', 'eight_puzzle.yaml'), ('narrow_corridor', 'narrow_corridor.yaml'),
                                     ('puzzle_dest_crash', 'puzzle_dest_crash.yaml')])
def test_facade_replays_reference_fixture(tag, cfg):
    if not gpu_available():
        pytest.skip('no GPU')
    from mfg_amd.factory import Factory
    rec, npz = G.load(tag, 0)
    random.seed(rec['py_seed'])
    env = Factory(cfg)
    assert env.named_action_space == rec['named_action_space']
    nl = env.spec.n_layers
    errs = []
    for r in rec['steps'][:700]:
        t = r['t']
        if r['step'] == 0:
            obs = list(env.reset().values())
        else:
            if r.get('crashed'):
                break
            _, obs, reward, done, info = env.step(list(r['actions']))
            if reward != r['reward'] or done != r['done']:
                errs.append((t, 'reward/done', reward, r['reward']))
            ok, bad = G.info_equal(info, r['info'])
            if not ok:
                errs.append((t, 'info', bad))
        if G.sha(G.obs_bytes([np.asarray(x)[:nl[a]] for a, x in enumerate(obs)])) != r['obs_sha']:
            errs.append((t, 'obs'))
        st = np.asarray(random.getstate()[1], dtype=np.uint32)
        if G.sha(st.tobytes()) != r['mt']:
            errs.append((t, 'python random state'))
        if len(errs) > 10:
            break
    env.close()
    assert not errs, errs[:10]


@pytest.mark.gpu
def test_batched_factory_matches_oracle():
    if not gpu_available():
        pytest.skip('no GPU')
    import torch
    import oracle as O
    from philox import synthetic_actions
    from mfg_amd.factory import BatchedFactory
    B, seed = 16, 3
    bf = BatchedFactory('rooms4.yaml', B, seed_base=100, obs_dtype='float64')
    obs = bf.reset()
    envs = [O.OracleEnv(bf.spec, 100 + i) for i in range(B)]
    ref = [e.reset() for e in envs]
    nl = bf.spec.n_layers
    for t in range(120):
        acts = synthetic_actions(seed, np.arange(B), t, bf.spec.n_actions)
        obs, rew, done, _ = bf.step(torch.tensor(acts))
        o, rw, dn = obs.cpu().numpy(), rew.cpu().numpy(), done.cpu().numpy()
        for i, e in enumerate(envs):
            r, d, _ = e.step(acts[i])
            assert list(rw[i]) == list(r) and bool(dn[i]) == d, (t, i)
            ro = e.reset() if d else e.obs_list()
            for a in range(bf.spec.n_agents):
                assert (o[i, a, :nl[a]] == ro[a]).all(), (t, i, a)
        if t == 5:
            info = bf.info(0, acts[0])
            assert info['step'] == t + 1
    bf.close()


@pytest.mark.gpu
@pytest.mark.parametrize('tag', ['simple1', 'rooms4', 'large8', 'alltest16', 'default_large'])
def test_facade_views_match_reference(tag):
    """summarize_state / summarize_header / render entities of the facade (engine record -> views) equal
    the reference's on the recorded actions, across episode resets (tools/gen_golden_views.py)."""
    if not gpu_available():
        pytest.skip('no GPU')
    import views_compare as V
    from mfg_amd.factory import Factory
    rec = V.load_views(tag)
    random.seed(rec['py_seed'])
    env = Factory(rec['config'])
    env.reset()
    steps = rec['steps']
    V.compare_record(env.spec, env.snapshot(), steps[0], f'{tag} reset')
    assert env.summarize_state() == V.summarize_state(env.spec, env.snapshot())
    for t, r in enumerate(steps[1:], 1):
        if r['actions'] is None:
            env.reset()
        else:
            env.step(r['actions'])
        V.compare_record(env.spec, env.snapshot(), V.expand(r, steps[0]), f'{tag} record {t}')
    env.close()


@pytest.mark.gpu
def test_facade_group_access_render_manual():
    if not gpu_available():
        pytest.skip('no GPU')
    from mfg_amd.factory import Factory
    env = Factory('large8.yaml', py_seed=3)  # not synced with Python's random: two independent envs
    env.reset()
    doors = env['Doors']
    assert doors.name == 'Doors' and len(doors) == env.spec.c.n_doors
    assert len(env['Agent']) == env.spec.n_agents
    assert env.render('rgb_array').shape == (env.spec.H, env.spec.W, 3)
    assert len(env.render('ansi').splitlines()) == env.spec.H
    # manual protocol == step on a twin env with the same seed
    twin = Factory('large8.yaml', py_seed=3)
    twin.reset()
    acts = [1] * env.spec.n_agents
    env.manual_step_init()
    res = [env.manual_agent_tick(f'Agent[{n}]', a) for n, a in zip(env.spec.agent_names, acts)]
    env.manual_finalize_init()
    rew, done, info = env.manual_step_finalize(None)
    _, obs2, rew2, done2, info2 = twin.step(acts)
    assert rew == rew2 and done == done2 and info == info2
    assert (env.manual_get_agent_obs(f'Agent[{env.spec.agent_names[0]}]') == obs2[0]).all()
    assert res[0].identifier == env.summarize_state()['agents'][0]['action']
    with pytest.raises(RuntimeError):
        env.manual_step_init()
        env.manual_agent_tick(f'Agent[{env.spec.agent_names[1]}]', 0)  # out of list order
    env.close()
    twin.close()

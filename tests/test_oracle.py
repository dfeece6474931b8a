"""CPU: the C oracle (test infrastructure) pinned against the reference.
  * RNG restatements vs CPython 3.10 `random` and numpy 2.2 PCG64 known answers (tests/golden/units.npz)
  * the spec compiler's ray table vs the reference RayCaster (units.npz)
  * full-episode replays of the reference's golden fixtures: rewards, done, info dict (through the host
    info rebuild), agent/door/battery state, global pos_dict, floor-list order, MT state, obs (f64)."""
import numpy as np
import pytest

import golden_compare as G

UNITS = np.load(G.GOLDEN / 'units.npz')
FIXTURES = [('large8', 'large8.yaml'), ('rooms4', 'rooms4.yaml'), ('simple1', 'simple1.yaml'),
            ('alltest16', 'alltest16.yaml'), ('default_large', 'default_large.yaml'),
            ('maint_rooms', 'maint_rooms.yaml'), ('grid128_64', 'grid128_64.yaml'),
            ('eight_puzzle', 'eight_puzzle.yaml'), ('narrow_corridor', 'narrow_corridor.yaml'),
            ('_obs_test', '_obs_test.yaml'), ('puzzle_dest_crash', 'puzzle_dest_crash.yaml'),
            ('corridor_quantity', 'corridor_quantity.yaml'), ('logic_stress', 'logic_stress.yaml'),
            ('clean_and_bring', 'clean_and_bring.yaml'), ('large_full', 'large_full.yaml'),
            ('grid128_r10', 'grid128_r10.yaml'), ('qquad_full', 'qquad_full.yaml'), ('grid128_r20', 'grid128_r20.yaml'),
            ('grid128_full', 'grid128_full.yaml'), ('wide40', 'wide40.yaml'),
            ('qquad_doors', 'qquad_doors.yaml'), ('agents81', 'agents81.yaml')]


def test_mt19937_matches_cpython():
    import oracle as O
    from mfg_amd.spec import seed_key
    assert (O.mt_u32_seq(seed_key(12345), 2000) == UNITS['mt_seed12345_first2000']).all()


@pytest.mark.parametrize('seed', [0, 1, 7, 2 ** 40 + 3])
@pytest.mark.parametrize('n', [2, 95, 120, 1077])
def test_shuffle_matches_cpython(seed, n):
    import oracle as O
    from mfg_amd.spec import seed_key
    x, nxt = O.mt_shuffle_range(seed_key(seed), n)
    assert (x == UNITS[f'shuffle_s{seed}_n{n}']).all()
    assert nxt == int(UNITS[f'shuffle_s{seed}_n{n}_next'][0])


def test_pcg64_uniform_matches_numpy():
    import oracle as O
    raw, uni = O.pcg_seq(69, 64, -0.2, 0.2)
    assert (raw[:16] == UNITS['pcg69_raw']).all()
    assert (uni == UNITS['pcg69_uniform']).all()


@pytest.mark.parametrize('r', [3, 4, 8])
def test_ray_table_matches_reference(r):
    from mfg_amd.spec import ray_table
    rays = ray_table(2 * r + 1)
    assert [len(x) for x in rays] == list(UNITS[f'rays_r{r}_len'])
    assert [p for ray in rays for pt in ray for p in pt] == list(UNITS[f'rays_r{r}_pts'])


@pytest.mark.parametrize('tag,cfg', FIXTURES)
@pytest.mark.parametrize('seed', [0, 1])
def test_oracle_replays_reference_fixture(tag, cfg, seed):
    import oracle as O
    from mfg_amd.spec import compile_spec
    from mfg_amd.info import rebuild_info, rebuild_rewards, step_results
    rec, npz = G.load(tag, seed)
    spec = compile_spec(cfg)
    env = O.OracleEnv(spec, rec['py_seed'])
    W = spec.W
    errs = []
    for r in rec['steps']:
        t, st = r['t'], r['step']
        if st == 0:
            obs = env.reset()
        else:
            rew, done, ev = env.step(r['actions'])
            obs = env.obs_list()
            if r.get('crashed'):
                assert ev.crashed
                continue
            if [float(x) for x in rew] != r['reward']:
                errs.append((t, 'reward'))
            # the host replay of the Result list (custom host rules merge into it) folds to the same f64 rewards
            if rebuild_rewards(spec, step_results(spec, r['actions'], ev)) != r['reward']:
                errs.append((t, 'host reward fold'))
            if done != r['done']:
                errs.append((t, 'done'))
            ok, bad = G.info_equal(rebuild_info(spec, r['actions'], ev, list(rew)), r['info'])
            if not ok:
                errs.append((t, 'info', bad))
        pos, bat, _ = env.agents()
        if [[int(p) // W, int(p) % W] for p in pos] != r['agent_pos']:
            errs.append((t, 'agent_pos'))
        if 'battery' in r and list(bat) != r['battery']:
            errs.append((t, 'battery'))
        if 'doors' in r:
            o_, tt = env.doors()
            if [[int(a), int(b)] for a, b in zip(o_, tt)] != [x[3:5] for x in r['doors']]:
                errs.append((t, 'doors'))
        pd = env.posdict()
        if G.posdict_sha(pd) != r['posdict_sha']:
            errs.append((t, 'posdict'))
        if 'posdict' in r and pd != {int(k): v for k, v in r['posdict'].items()}:
            errs.append((t, 'posdict dump'))
        if G.sha(env.floor().tobytes()) != r['floor_sha']:
            errs.append((t, 'floor order'))
        if G.sha(env.mt_state().tobytes()) != r['mt']:
            errs.append((t, 'mt state'))
        pc = env.pcg_state()
        if str((int(pc[0]) << 64) | int(pc[1])) != r['pcg']:
            errs.append((t, 'pcg state'))
        if G.sha(G.obs_bytes(obs)) != r['obs_sha']:
            errs.append((t, 'obs'))
        if len(errs) > 10:
            break
    env.close()
    assert not errs, errs[:10]


def test_fixture_negative_control():
    """A wrong seed must NOT reproduce the fixture (guards against a vacuous comparison)."""
    import oracle as O
    from mfg_amd.spec import compile_spec
    rec, _ = G.load('large8', 0)
    spec = compile_spec('large8.yaml')
    env = O.OracleEnv(spec, rec['py_seed'] + 1)
    env.reset()
    pos, _, _ = env.agents()
    W = spec.W
    assert [[int(p) // W, int(p) % W] for p in pos] != rec['steps'][0]['agent_pos']

"""CPU: the host-side entity views (`mfg_amd.views`: Factory.summarize_state / summarize_header /
state.entities.render, factory.py:262-292) against the reference's own outputs, recorded by
tools/gen_golden_views.py, with the C oracle (test infrastructure) providing the state."""
import pytest

import views_compare as V


@pytest.mark.parametrize('tag', V.VIEW_FIXTURES)
def test_views_match_reference(tag):
    import oracle as O
    from mfg_amd.spec import compile_spec
    rec = V.load_views(tag)
    spec = compile_spec(rec['config'])
    env = O.OracleEnv(spec, rec['py_seed'])
    env.reset()
    steps = rec['steps']
    V.compare_record(spec, V.oracle_snapshot(env), steps[0], f'{tag} reset')
    for t, r in enumerate(steps[1:], 1):
        if r['actions'] is None:  # the reference reset after a done step
            env.reset()
        else:
            env.step(r['actions'], with_obs=False)
        V.compare_record(spec, V.oracle_snapshot(env), V.expand(r, steps[0]), f'{tag} record {t}')
    env.close()


def test_views_negative_control():
    import oracle as O
    from mfg_amd.spec import compile_spec
    rec = V.load_views('large8')
    spec = compile_spec(rec['config'])
    env = O.OracleEnv(spec, rec['py_seed'] + 1)  # another seed: other positions
    env.reset()
    with pytest.raises(AssertionError):
        V.compare_record(spec, V.oracle_snapshot(env), rec['steps'][0], 'wrong seed')
    env.close()


def test_group_view_and_ansi():
    import oracle as O
    from mfg_amd.spec import compile_spec
    from mfg_amd import views
    spec = compile_spec('large8.yaml')
    env = O.OracleEnv(spec, 0)
    env.reset()
    snap = V.oracle_snapshot(env)
    doors = views.group_view(spec, snap, 'Doors')
    assert doors.name == 'Doors' and len(doors) == spec.c.n_doors and doors[0]['state'] == 'closed'
    assert len(views.group_view(spec, snap, 'Agent')) == spec.n_agents
    with pytest.raises(KeyError):
        views.group_view(spec, snap, 'NoSuchGroup')
    frame = views.render_ansi(spec, snap).splitlines()
    assert len(frame) == spec.H and all(len(r) == spec.W for r in frame)
    assert sum(r.count('A') + r.count('!') for r in frame) >= 1
    env.close()

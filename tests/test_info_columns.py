"""Batched info columns: the device-side evaluation of the reference's info dict for all B
envs equals the per-env host rebuild (info.rebuild_info, itself pinned by the reference fixtures), key set and
f64 values, on every config with rule results of every kind."""
import numpy as np
import pytest

from conftest import gpu_available


def test_columns_cover_the_rebuild_keys_on_cpu():
    """CPU: on recorded reference events the columns' key set contains every key the fixtures' info dicts use."""
    import golden_compare as G
    from mfg_amd.spec import compile_spec
    from mfg_amd.info_columns import InfoColumns
    for tag in ['large8', 'rooms4', 'alltest16', 'eight_puzzle', 'puzzle_dest_crash', 'maint_rooms']:
        spec = compile_spec(f'{tag}.yaml')
        cols = InfoColumns(spec)
        rec, _ = G.load(tag, 0)
        seen = set()
        for r in rec['steps']:
            if r.get('info'):
                seen |= {k for k in r['info'] if not k.startswith('Maintainer[')}
        assert seen <= set(cols.columns), (tag, sorted(seen - set(cols.columns)))


@pytest.mark.gpu
@pytest.mark.parametrize('cfg,B,steps', [('large8.yaml', 256, 40), ('rooms4.yaml', 256, 120), ('alltest16.yaml', 64, 40),
                                         ('maint_rooms.yaml', 64, 60), ('eight_puzzle.yaml', 128, 60),
                                         ('puzzle_dest_crash.yaml', 64, 60), ('corridor_quantity.yaml', 64, 60)])
def test_info_columns_equal_host_rebuild(cfg, B, steps):
    if not gpu_available():
        pytest.skip('no GPU')
    import torch
    from philox import synthetic_actions
    from mfg_amd.factory import BatchedFactory
    from mfg_amd.engine import events_from_rows
    from mfg_amd.info import rebuild_info
    bf = BatchedFactory(cfg, B, seed_base=40)
    bf.reset()
    checked = 0
    for t in range(steps):
        acts = synthetic_actions(11, np.arange(B), t, bf.spec.n_actions)
        at = torch.tensor(acts, device=bf.device)
        bf.step(at)
        names, vals, pres = bf.info_columns(at)
        ea, ew, em = bf.ev_act.cpu().numpy(), bf.ev_watch.cpu().numpy(), bf.ev_misc.cpu().numpy()
        rw = bf.reward.cpu().numpy()
        for b in range(0, B, max(1, B // 32)):
            ev = events_from_rows(ea[b], ew[b], em[b])
            if ev['crashed']:
                continue
            want = rebuild_info(bf.spec, acts[b], ev, [float(x) for x in rw[b]])
            got = bf._info_cols.to_dict(vals, pres, b, maint_base=ev['maint_base'])
            assert got == want, (cfg, t, b, sorted(set(got.items()) ^ set(want.items()))[:6])
            checked += 1
    bf.close()
    assert checked > 0

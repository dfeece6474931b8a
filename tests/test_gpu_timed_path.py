"""GPU parity of the exact mode bench.py times:
  * mfg_step with K=8 fused steps, Philox actions (actions=None), f64 obs (the headline line since round 4, the
    reference's own obs precision) and float32 obs (its side line), auto-reset, at the headline batch B=65536 on
    large8 (C3), for 608 steps (across the 500-step episode boundary). 256 envs spread over the batch (incl. 0
    and B-1) are checked every step against their own C-oracle env: f64 rewards with ==, done, the event rows,
    obs bit-equal to the oracle's f64 obs (cast to float32 for the f32 mode), and after every call (one k_replay
    each) the MT19937 state and floor order.
  * K=8 and K=1 calls give identical outputs and identical state (the cross-call shuffle-debt carry and the
    per-k output offsets), on large8 and on the step-RNG paths (dirt respawn, maintainers).
  * the documented row widths of include/mfg.h: guard words after every output buffer stay untouched.
  * sharding: two engines over [0, B/2) and [B/2, B) with env_base/seed_base offsets == one engine over B.
"""
import hashlib

import numpy as np
import pytest

from conftest import gpu_available
from mfg_amd.engine import EV_MISC

pytestmark = pytest.mark.gpu


def _engine(cfg, B, **kw):
    if not gpu_available():
        pytest.skip('no GPU')
    import torch
    from mfg_amd.spec import compile_spec
    from mfg_amd.engine import Engine
    spec = compile_spec(cfg)
    return torch, spec, Engine(spec, B, **kw)


def _buffers(torch, eng, K, obs_dtype):
    B, A, dev = eng.B, eng.A, eng.device
    return dict(obs=torch.zeros((K,) + eng.obs_shape(), dtype=obs_dtype, device=dev),
                reward=torch.zeros((K, B, A), dtype=torch.float64, device=dev),
                done=torch.zeros((K, B), dtype=torch.uint8, device=dev),
                ev_act=torch.zeros((K, B, A), dtype=torch.uint8, device=dev),
                ev_watch=torch.zeros((K, B, A), dtype=torch.uint8, device=dev),
                ev_misc=torch.zeros((K, B, EV_MISC), dtype=torch.int32, device=dev))


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


@pytest.mark.timeout(900)
def test_timed_path_k8_fp32_b65536_matches_oracle():
    _timed_path(np.float32)


@pytest.mark.timeout(900)
def test_timed_path_k8_f64_b65536_matches_oracle():
    _timed_path(np.float64)


def _timed_path(odt):
    import oracle as O
    from philox import synthetic_actions
    from mfg_amd.engine import RecordView, events_from_rows
    B, K, calls, base, pseed = 65536, 8, 76, 0, 12345
    torch, spec, eng = _engine('large8.yaml', B)
    A, nl = spec.n_agents, spec.n_layers
    rng = np.random.default_rng(3)
    idx = np.unique(np.concatenate([[0, 1, B // 2, B - 2, B - 1], rng.choice(B, 251, replace=False)]))
    idx_t = torch.as_tensor(idx, device=eng.device)
    buf = _buffers(torch, eng, K, torch.float32 if odt == np.float32 else torch.float64)
    ubits = np.uint32 if odt == np.float32 else np.uint64
    eng.reset(obs=buf['obs'][0], init=True, seed_base=base)
    envs = [O.OracleEnv(spec, base + int(i)) for i in idx]
    o0 = buf['obs'][0][idx_t].cpu().numpy()
    for j, env in enumerate(envs):
        ro = env.reset()
        for a in range(A):
            assert (o0[j, a, :nl[a]] == ro[a].astype(odt)).all(), f'reset obs env {idx[j]} agent {a}'
    ndone = 0
    step = 0
    for c in range(calls):
        eng.step(K, actions=None, philox_seed=pseed, env_base=0, step_base=step, auto_reset=True, **buf)
        rw = buf['reward'][:, idx_t].cpu().numpy()
        dn = buf['done'][:, idx_t].cpu().numpy()
        ob = buf['obs'][:, idx_t].cpu().numpy()
        ea = buf['ev_act'][:, idx_t].cpu().numpy()
        ew = buf['ev_watch'][:, idx_t].cpu().numpy()
        em = buf['ev_misc'][:, idx_t].cpu().numpy()
        for k in range(K):
            acts = synthetic_actions(pseed, idx, step + k, spec.n_actions)
            for j, env in enumerate(envs):
                r_ref, d_ref, ev_ref = env.step(acts[j])
                tag = f'call {c} k {k} env {idx[j]}'
                assert list(rw[k, j]) == list(r_ref), f'{tag} reward {rw[k, j]} vs {r_ref}'
                assert bool(dn[k, j]) == d_ref, f'{tag} done'
                ev = events_from_rows(ea[k, j], ew[k, j], em[k, j])
                assert ev['act'] == list(ev_ref.act[:A]) and ev['watch'] == list(ev_ref.watch[:A]), f'{tag} events'
                assert ev['door_coll'] == ev_ref.door_coll and ev['door_coll_hi'] == ev_ref.door_coll_hi, f'{tag} events'
                assert ev['done_mask'] == ev_ref.done_mask, f'{tag} events'
                assert ev['step'] == ev_ref.step, f'{tag} step'
                if d_ref:
                    ndone += 1
                    ro = env.reset()
                else:
                    ro = env.obs_list()
                for a in range(A):
                    want = ro[a].astype(odt)
                    got = ob[k, j, a, :nl[a]]
                    if not (got.view(ubits) == want.view(ubits)).all():
                        dif = np.argwhere(got != want)
                        raise AssertionError(f'{tag} agent {a} {odt.__name__} obs: {len(dif)} diffs, first '
                                             f'{[(tuple(x), got[tuple(x)], want[tuple(x)]) for x in dif[:4]]}')
        step += K
        # after the call's k_replay: RNG state and floor order of the sampled envs
        st = eng.export_state()[idx_t].cpu().numpy()
        for j, env in enumerate(envs):
            rv = RecordView(st[j], eng.layout, spec)
            assert _sha(rv.mt()) == _sha(env.mt_state()), f'call {c} env {idx[j]} MT state'
            assert _sha(rv.perm()) == _sha(env.floor()), f'call {c} env {idx[j]} floor order'
    eng.close()
    assert step > 500 and ndone == len(idx)  # every sampled env crossed the step-500 episode boundary


@pytest.mark.timeout(900)
def test_timed_path_k8_b65536_final_state_of_16384_envs(full=False):
    """the benched mode (K = 8, Philox actions, f64 obs, auto-reset, B = 65,536, 608 steps across the
    step-500 mass reset, where every env goes through the done list at once) checked against the C oracle's own rollout
    of the same envs (oracle/oracle.py rollout: the C loop, blocks in threads) on 16,384 envs (16 blocks of 1,024 spread
    over the batch, env 0 and B - 1 included; full=True: every env, ~40M oracle env-steps, 165 s on the test box,
    profiles/r05m_final_state_all_65536_envs.txt): per env the f64 reward sum of every agent (added step by step on both
    sides, so ==), the number of episode ends, and the final MT19937 state, index and floor order. (The per-step obs,
    rewards and events of 256 of these envs are compared in the tests above.) The default keeps the test well under a
    minute: the harness takes a command silent for 3 minutes as hung."""
    import oracle as O
    B, K, calls, pseed = 65536, 8, 76, 12345
    torch, spec, eng = _engine('large8.yaml', B)
    buf = _buffers(torch, eng, K, torch.float64)
    eng.reset(obs=buf['obs'][0], init=True, seed_base=0)
    rsum = torch.zeros((B, spec.n_agents), dtype=torch.float64, device=eng.device)
    ndone = torch.zeros(B, dtype=torch.int32, device=eng.device)
    for c in range(calls):
        eng.step(K, actions=None, philox_seed=pseed, env_base=0, step_base=c * K, auto_reset=True, **buf)
        for k in range(K):  # the oracle adds step by step: the same f64 additions in the same order
            rsum += buf['reward'][k]
            ndone += buf['done'][k].to(torch.int32)
    st = eng.export_state().cpu().numpy()
    rs, nd = rsum.cpu().numpy(), ndone.cpu().numpy()
    eng.close()
    lay, nf = eng.layout, spec.c.n_floor
    blocks = [(k * 4096, 4096) for k in range(B // 4096)] if full else \
        [(k * 4096 + (3072 if k == 15 else 0), 1024) for k in range(B // 4096)]
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(len(blocks)) as ex:
        res = list(ex.map(lambda b: O.rollout(spec, 0, b[0], b[1], calls * K, pseed, threads=1), blocks))
    for (s0, n), (rw, dn, mt, fl) in zip(blocks, res):
        sl = slice(s0, s0 + n)
        rec = st[sl]
        g_mt = rec[:, lay['o_mt']:lay['o_mt'] + 4 * 624].copy().view(np.uint32)
        g_idx = rec[:, lay['o_hdr']:lay['o_hdr'] + 160].copy().view(np.int32)[:, 6]  # H_MT_IDX
        g_fl = rec[:, lay['o_perm']:lay['o_perm'] + 2 * nf].copy().view(np.uint16).astype(np.int32)
        bad = np.nonzero((rs[sl] != rw).any(1) | (nd[sl] != dn) | (g_mt != mt[:, :624]).any(1) |
                         (g_idx != mt[:, 624].astype(np.int32)) | (g_fl != fl).any(1))[0]
        assert not len(bad), f'{len(bad)} envs differ from the oracle, first env {s0 + int(bad[0])}'
        assert (dn >= 1).all()  # every checked env crossed the step-500 episode boundary
    assert sum(n for _, n in blocks) == (B if full else B // 4)


@pytest.mark.parametrize('cfg,B,steps', [('large8.yaml', 4096, 80), ('rooms4.yaml', 2048, 120),
                                         ('maint_rooms.yaml', 256, 96), ('alltest16.yaml', 512, 64)])
def test_fused_k8_equals_k1(cfg, B, steps):
    """Same envs, same Philox actions: eight K=1 calls and one K=8 call produce bit-identical outputs and
    state (obs f32 here, the bench's dtype)."""
    torch, spec, e1 = _engine(cfg, B)
    _, _, e8 = _engine(cfg, B)
    b1 = _buffers(torch, e1, 1, torch.float32)
    b8 = _buffers(torch, e8, 8, torch.float32)
    e1.reset(obs=b1['obs'][0], init=True, seed_base=70)
    e8.reset(obs=b8['obs'][0], init=True, seed_base=70)
    assert torch.equal(b1['obs'][0], b8['obs'][0])
    for t0 in range(0, steps, 8):
        e8.step(8, actions=None, philox_seed=9, step_base=t0, auto_reset=True, **b8)
        for k in range(8):
            e1.step(1, actions=None, philox_seed=9, step_base=t0 + k, auto_reset=True, **b1)
            for name in b1:
                assert torch.equal(b1[name][0], b8[name][k]), f'{cfg} step {t0 + k} {name}'
        assert torch.equal(e1.export_state(), e8.export_state()), f'{cfg} state after step {t0 + 7}'
    e1.close()
    e8.close()


@pytest.mark.parametrize('cfg,B,steps', [('large8.yaml', 2048, 64), ('alltest16.yaml', 512, 64)])
def test_deferred_replay_equals_per_call_replay(cfg, B, steps):
    """MFG_STEP_DEFER_REPLAY on seven of every eight K=1 calls (the replay then runs on the eighth): every output
    of every step and the state after each eighth call equal one K=8 call (include/mfg.h: the debt is paid before
    anything consumes the floor order; alltest16's RespawnDirt consumes it inside a step)."""
    torch, spec, e1 = _engine(cfg, B)
    _, _, e8 = _engine(cfg, B)
    b1 = _buffers(torch, e1, 1, torch.float32)
    b8 = _buffers(torch, e8, 8, torch.float32)
    e1.reset(obs=b1['obs'][0], init=True, seed_base=71)
    e8.reset(obs=b8['obs'][0], init=True, seed_base=71)
    for t0 in range(0, steps, 8):
        e8.step(8, actions=None, philox_seed=5, step_base=t0, auto_reset=True, **b8)
        for k in range(8):
            e1.step(1, actions=None, philox_seed=5, step_base=t0 + k, auto_reset=True, defer_replay=k < 7, **b1)
            for name in b1:
                assert torch.equal(b1[name][0], b8[name][k]), f'{cfg} step {t0 + k} {name}'
        assert torch.equal(e1.export_state(), e8.export_state()), f'{cfg} state after step {t0 + 7}'
    e1.close()
    e8.close()


def test_output_rows_respect_header_widths():
    """Every output buffer sized exactly as include/mfg.h documents ([K][B][A], [K][B], [K][B][MFG_EV_MISC_N],
    [K][B][A][lmax][d][d]) followed by guard words: the engine writes every row and nothing past the end."""
    torch, spec, eng = _engine('alltest16.yaml', 37)
    K, B, A = 3, eng.B, eng.A
    G = 4096
    sentinel = 0x5A
    shapes = dict(reward=(K * B * A * 8), done=(K * B), ev_act=(K * B * A), ev_watch=(K * B * A),
                  ev_misc=(K * B * EV_MISC * 4), obs=(K * B * A * eng.lmax * eng.obs_hw[0] * eng.obs_hw[1] * 4))
    raw = {k: torch.full((n + G,), sentinel, dtype=torch.uint8, device=eng.device) for k, n in shapes.items()}
    views = dict(reward=raw['reward'][:shapes['reward']].view(torch.float64),
                 done=raw['done'][:shapes['done']], ev_act=raw['ev_act'][:shapes['ev_act']],
                 ev_watch=raw['ev_watch'][:shapes['ev_watch']],
                 ev_misc=raw['ev_misc'][:shapes['ev_misc']].view(torch.int32),
                 obs=raw['obs'][:shapes['obs']].view(torch.float32))
    eng.reset(init=True, seed_base=5)
    eng.step(K, actions=None, philox_seed=1, step_base=0, auto_reset=True, **views)
    torch.cuda.synchronize()
    for k, n in shapes.items():
        assert (raw[k][n:] == sentinel).all(), f'{k}: write past the documented row width'
    misc = views['ev_misc'].view(K, B, EV_MISC).cpu().numpy()
    dn = views['done'].view(K, B).cpu().numpy()
    assert (dn <= 1).all()
    # every ev_misc row carries its step: 1 after the reset, +1 per step, 1 again after an auto-reset
    assert (misc[0, :, 8] == 1).all()
    for k in range(1, K):
        assert (misc[k, :, 8] == np.where(dn[k - 1] == 1, 1, misc[k - 1, :, 8] + 1)).all(), f'row {k} step'
    ok = (misc[:, :, 6] & 2) == 0  # rows of envs that did not crash (a crash stops the agent loop)
    acted = (views['ev_act'].view(K, B, A).cpu().numpy() & 0x80) != 0
    assert ok.any() and acted[ok].all(), 'every agent of a non-crashed env acted in every row'
    eng.close()


@pytest.mark.parametrize('cfg,B,steps', [('large8.yaml', 64, 96), ('rooms4.yaml', 64, 96)])
def test_two_shards_equal_one_engine(cfg, B, steps):
    """shard s owns global envs [s*B/2, (s+1)*B/2), seeded seed_base + global index, Philox keyed
    on the global index (env_base). Two shard engines reproduce one engine over all B envs bit-exactly."""
    torch, spec, full = _engine(cfg, B)
    half = B // 2
    shards = [_engine(cfg, half)[2] for _ in range(2)]
    bf = _buffers(torch, full, 1, torch.float32)
    bs = [_buffers(torch, s, 1, torch.float32) for s in shards]
    full.reset(obs=bf['obs'][0], init=True, seed_base=300)
    for i, s in enumerate(shards):
        s.reset(obs=bs[i]['obs'][0], init=True, seed_base=300 + i * half)
    for t in range(steps):
        full.step(1, actions=None, philox_seed=4, env_base=0, step_base=t, auto_reset=True, **bf)
        for i, s in enumerate(shards):
            s.step(1, actions=None, philox_seed=4, env_base=i * half, step_base=t, auto_reset=True, **bs[i])
        for name in bf:
            joined = torch.cat([bs[0][name][0], bs[1][name][0]], dim=0)
            assert torch.equal(joined, bf[name][0]), f'{cfg} step {t} {name}'
    st = full.export_state()
    assert torch.equal(torch.cat([shards[0].export_state(), shards[1].export_state()]), st)
    for e in [full] + shards:
        e.close()


@pytest.mark.parametrize('auto_reset', [False, True])
def test_out_of_range_action_crashes_only_that_env(auto_reset):
    """An action index outside [0, n_actions[a]) is the reference's IndexError (factory.py:201-206): that env
    reports MFG_CRASH_ACTION + done and takes no step; every other env steps exactly like the oracle. With
    auto-reset the crashed env is reset and steps normally afterwards."""
    import oracle as O
    from mfg_amd import abi
    B = 8  # noqa: N806
    torch, spec, eng = _engine('large8.yaml', B)
    A = spec.n_agents
    buf = _buffers(torch, eng, 1, torch.float64)
    eng.reset(obs=buf['obs'][0], init=True, seed_base=0)
    envs = [O.OracleEnv(spec, i) for i in range(B)]
    for e in envs:
        e.reset()
    rng = np.random.default_rng(5)
    # agent 0: nothing acts before the IndexError, so a reset env matches a fresh oracle reset (agents ahead of a
    # bad index do act first, as in the reference's ordered loop, which the oracle does not model)
    bad = {3: (0, spec.n_actions[0]), 5: (0, -1)}
    for t in range(3):
        acts = np.stack([rng.integers(0, spec.n_actions[a], size=B) for a in range(A)], 1).astype(np.int32)
        if t == 0:
            for env, (a, v) in bad.items():
                acts[env, a] = v
        eng.step(1, actions=torch.as_tensor(acts, device=eng.device), reward=buf['reward'], done=buf['done'],
                 obs=buf['obs'], ev_act=buf['ev_act'], ev_watch=buf['ev_watch'], ev_misc=buf['ev_misc'],
                 auto_reset=auto_reset)
        rew, done = buf['reward'][0].cpu().numpy(), buf['done'][0].cpu().numpy()
        flags = buf['ev_misc'][0, :, abi.EVM_FLAGS].cpu().numpy()
        for i in range(B):
            crashed_now = t == 0 and i in bad
            if crashed_now or (t > 0 and i in bad and not auto_reset):
                assert done[i] == 1 and (flags[i] >> 1) & 1, (t, i)
                assert (flags[i] >> 8) & 0xFF == 8  # MFG_CRASH_ACTION (include/mfg.h)
                continue
            r, d, _ = envs[i].step(acts[i])
            assert list(rew[i]) == list(r) and bool(done[i]) == bool(d), (t, i)
            assert not (flags[i] >> 1) & 1, (t, i)
        if t == 0 and auto_reset:
            for i in bad:  # the engine reset them after the crash: the oracle does the same
                envs[i].reset()
    eng.close()

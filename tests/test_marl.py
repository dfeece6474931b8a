"""On-GPU MARL over packed observations (mfg_amd/marl.py).

CPU: the learner (RecurrentAC fed by packed obs through embedding_bag + the A2C loss) against golden vectors
produced by the reference's own network and loss (tests/golden/marl_a2c.npz, tools/gen_golden_marl.py:
algorithms/marl/networks.py RecurrentAC, algorithms/marl/base_ac.py actor_critic/learn). f32 arithmetic in a
different summation order: loss and gradients within 1e-5 relative (+1e-7 absolute), weights after one
RMSprop step within 1e-6 absolute.
GPU: the engine's packed rows scatter back to the dense f32 obs bit-exactly, its fused projection matches a
torch f64 GEMM of the dense obs within 1e-5 relative, and the A2C loop trains on the device.
"""
from pathlib import Path

import numpy as np
import pytest
import torch

from mfg_amd.marl import RecurrentAC, a2c_loss

GOLD = Path(__file__).resolve().parent / 'golden' / 'marl_a2c.npz'


def pack(obs, cap):
    """Dense [N, T, ...] -> (idx u16, val f32) [N, T, cap] of the nonzero entries of obs.float()."""
    flat = torch.as_tensor(obs).reshape(obs.shape[0], obs.shape[1], -1).float()
    N, T, K = flat.shape
    idx = torch.zeros((N, T, cap), dtype=torch.uint16)
    val = torch.zeros((N, T, cap), dtype=torch.float32)
    for n in range(N):
        for t in range(T):
            nz = torch.nonzero(flat[n, t]).flatten()
            assert len(nz) <= cap
            idx[n, t, :len(nz)] = nz.to(torch.uint16)
            val[n, t, :len(nz)] = flat[n, t, nz]
    return idx, val


def load_case(z, i):
    c = {k.split('.', 1)[1]: z[k] for k in z.files if k.startswith(f'c{i}.')}
    st = {k[2:]: torch.from_numpy(v) for k, v in c.items() if k.startswith('w.')}
    N, T1 = c['actions'].shape
    obs_shape = c['obs'].shape[2:]
    net = RecurrentAC(observation_size=obs_shape, n_actions=int(c['n_actions']),
                      obs_emb_size=st['obs_proj.weight'].shape[0], action_emb_size=st['action_emb.weight'].shape[1],
                      hidden_size_actor=st['gru_actor.weight_hh_l0'].shape[1],
                      hidden_size_critic=st['gru_critic.weight_hh_l0'].shape[1], n_agents=N,
                      use_agent_embedding=bool(c['use_agent_embedding']))
    net.load_state_dict(st)
    return c, net


@pytest.mark.parametrize('i', [0, 1, 2])
def test_a2c_learner_matches_reference(i):
    z = np.load(GOLD)
    c, net = load_case(z, i)
    N = c['actions'].shape[0]
    idx, val = pack(c['obs'], cap=64)
    acts = torch.from_numpy(c['actions']).long()
    emb = net.project_packed(idx, val)
    out = net.forward_emb(emb, acts, torch.from_numpy(c['ha0']), torch.from_numpy(c['hc0']),
                          agent_ids=torch.arange(N))
    loss = a2c_loss(out, acts, torch.from_numpy(c['reward'])[:, 1:], torch.from_numpy(c['done'])[:, 1:],
                    gamma=0.99, entropy_coef=0.01, vf_coef=0.5, gae_coef=float(c['gae_coef']))
    ref = float(c['loss'])
    assert abs(loss.item() - ref) <= 1e-5 * abs(ref) + 1e-7, (loss.item(), ref)
    opt = torch.optim.RMSprop(net.parameters(), lr=3e-4, eps=1e-5)
    opt.zero_grad()
    loss.backward()
    for k, p in net.named_parameters():
        g = p.grad if p.grad is not None else torch.zeros_like(p)
        gr = torch.from_numpy(c['g.' + k])
        assert torch.allclose(g, gr, rtol=1e-4, atol=1e-6), (k, (g - gr).abs().max())
    torch.nn.utils.clip_grad_norm_(net.parameters(), 0.5)
    opt.step()
    for k, p in net.named_parameters():
        assert torch.allclose(p.detach(), torch.from_numpy(c['a.' + k]), rtol=0, atol=1e-6), k


def test_dense_forward_is_the_reference_forward():
    """The reference-signature forward (dense obs) equals the packed path on the same inputs."""
    z = np.load(GOLD)
    c, net = load_case(z, 0)
    acts = torch.from_numpy(c['actions']).long()
    ha, hc = torch.from_numpy(c['ha0']), torch.from_numpy(c['hc0'])
    dense = net(torch.from_numpy(c['obs']), acts, ha, hc)
    idx, val = pack(c['obs'], cap=64)
    packed = net.forward_emb(net.project_packed(idx, val), acts, ha, hc)
    for k in ('logits', 'critic'):
        assert torch.allclose(dense[k], packed[k], rtol=1e-5, atol=1e-6), k


def test_stepwise_restarts():
    """starts=all-False equals one GRU call; a start at entry s equals a fresh run from s with zero state."""
    torch.manual_seed(0)
    net = RecurrentAC((3, 4, 4), 5, 16, 4, 8, 8, 3, use_agent_embedding=False)
    N, T = 3, 6
    emb = torch.randn(N, T, 16)
    acts = torch.randint(-1, 5, (N, T))
    h = torch.randn(N, 1, 8)
    full = net.forward_emb(emb, acts, h, h)
    st = net.forward_emb(emb, acts, h, h, starts=torch.zeros(N, T, dtype=torch.bool))
    assert torch.allclose(full['logits'], st['logits'], atol=1e-6)
    starts = torch.zeros(N, T, dtype=torch.bool)
    starts[:, 3] = True
    r = net.forward_emb(emb, acts, h, h, starts=starts)
    fresh = net.forward_emb(emb[:, 3:], acts[:, 3:], torch.zeros_like(h), torch.zeros_like(h))
    assert torch.allclose(r['logits'][:, 3:], fresh['logits'], atol=1e-6)
    assert torch.allclose(r['critic'][:, :3], full['critic'][:, :3], atol=1e-6)


# ---------------------------------------------------------------------------------------------------------
# GPU: the engine's packed mode
# ---------------------------------------------------------------------------------------------------------
def _engine_pair(cfg, B, K, E=96, cap=64, seed_base=0, proj=True):
    from mfg_amd.spec import compile_spec
    from mfg_amd.engine import Engine, PackedObs
    spec = compile_spec(cfg)
    dense, packed = Engine(spec, B, device=0), Engine(spec, B, device=0)
    kdim = dense.lmax * dense.obs_hw[0] * dense.obs_hw[1]
    g = torch.Generator().manual_seed(1)
    w = (torch.randn(E, kdim, generator=g) * 0.1).cuda() if proj else None
    b = (torch.randn(E, generator=g) * 0.1).cuda() if proj else None
    po = PackedObs(packed, K=K, cap=cap, weight=w, bias=b)  # no weight: the entries-only render
    return spec, dense, packed, po, w, b


def _check_rows(dense_obs, po, w, b, k, block_order=False):
    """Packed row k == dense f32 obs bit-exactly; emb == f64 GEMM within 1e-5 relative. Stored entries in ascending
    flat index order, or with block_order (renders with rays of more than 12 points) in (64-cell block, layer, cell)
    order (include/mfg.h)."""
    B, A = dense_obs.shape[:2]
    flat = dense_obs.reshape(B, A, -1)
    nnz = (flat != 0).sum(-1).to(torch.int32)
    assert torch.equal(po.count[k], nnz)
    assert torch.equal(po.dense(k).reshape(B, A, -1), flat)
    if po.idx is not None:
        ix = po.idx[k].long()
        if block_order:
            dd = dense_obs.shape[-2] * dense_obs.shape[-1]
            ix = (ix % dd) // 64 * flat.shape[-1] + ix
        n = torch.clamp(po.count[k], max=po.cap).unsqueeze(-1)
        later = torch.arange(1, po.cap, device=ix.device) < n
        assert bool(((ix[..., 1:] > ix[..., :-1]) | ~later).all())
    if w is None:
        return
    ref = flat.double() @ w.double().t() + b.double()
    err = (po.emb[k].double() - ref).abs()
    tol = 1e-5 * (flat.double().abs() @ w.double().abs().t() + b.double().abs()) + 1e-6
    assert bool((err <= tol).all()), float(err.max())


@pytest.mark.gpu
@pytest.mark.parametrize('cfg,B,K,proj', [('large8.yaml', 2048, 8, True), ('rooms4.yaml', 512, 4, True),
                                          ('alltest16.yaml', 96, 2, True), ('simple1.yaml', 256, 4, True),
                                          ('large8.yaml', 2048, 8, False), ('alltest16.yaml', 96, 2, False),
                                          ('grid128_64.yaml', 8, 2, False)])
def test_packed_obs_matches_dense(cfg, B, K, proj):
    spec, dense, packed, po, w, b = _engine_pair(cfg, B, K, proj=proj, cap=1024 if 'grid128' in cfg else 64)
    obs = torch.zeros(dense.obs_shape(K), dtype=torch.float32, device='cuda')
    dense.reset(obs=obs[0], init=True, seed_base=5)
    packed.reset(obs=po.view(0), init=True, seed_base=5)
    _check_rows(obs[0], po, w, b, 0, block_order='grid128' in cfg)
    for it in range(3):
        dense.step(K, philox_seed=9, step_base=1 + it * K, obs=obs, auto_reset=True)
        packed.step(K, philox_seed=9, step_base=1 + it * K, obs=po, auto_reset=True)
        for k in range(K):
            _check_rows(obs[k], po, w, b, k, block_order='grid128' in cfg)
    dense.close()
    packed.close()


@pytest.mark.gpu
def test_packed_cap_truncation_is_reported():
    spec, dense, packed, po, w, b = _engine_pair('large8.yaml', 256, 1, cap=2)
    obs = torch.zeros(dense.obs_shape(1), dtype=torch.float32, device='cuda')
    dense.reset(obs=obs[0], init=True)
    packed.reset(obs=po, init=True)
    flat = obs[0].reshape(256, spec.n_agents, -1)
    assert torch.equal(po.count[0], (flat != 0).sum(-1).to(torch.int32))
    # a truncated row keeps its first cap entries in flat index order
    pos = torch.arange(flat.shape[-1], device=flat.device).expand_as(flat)
    first = torch.where(flat != 0, pos, flat.shape[-1]).sort(-1).values[..., :2]
    full = po.count[0] >= 2
    assert torch.equal(po.idx[0].long()[full], first[full])
    # the projection covers all entries even when the stored row is truncated
    ref = flat.double() @ w.double().t() + b.double()
    assert float((po.emb[0].double() - ref).abs().max()) < 1e-3
    with pytest.raises(RuntimeError):
        po.check()


@pytest.mark.gpu
def test_batched_a2c_trains_on_device():
    from mfg_amd.factory import BatchedFactory
    from mfg_amd.marl import BatchedA2C
    f = BatchedFactory('large8.yaml', 512, seed_base=3)
    tr = BatchedA2C(f, n_steps=5, generator=torch.Generator(device='cuda').manual_seed(0))
    w0 = tr.net.obs_proj.weight.detach().clone()
    loss = tr.train(4)
    assert tr.updates == 4 and torch.isfinite(loss)
    assert not torch.equal(w0, tr.net.obs_proj.weight.detach())
    # after the updates the engine projects with the new weights: emb of o_0 == embedding_bag of its entries
    e = tr.net.project_packed(tr.pobs.idx[0], tr.pobs.val[0])
    assert torch.allclose(e, tr.pobs.emb[0], rtol=1e-5, atol=1e-5)
    # one more step renders with the refreshed weights inside the kernel
    tr.step()
    e1 = tr.net.project_packed(tr.pobs.idx[1], tr.pobs.val[1])
    assert torch.allclose(e1, tr.pobs.emb[1], rtol=1e-5, atol=1e-5)
    f.close()


@pytest.mark.gpu
def test_batched_a2c_graph_update_matches_eager():
    """graph=True (the update captured once as a HIP graph after two eager warm-up updates, then replayed) trains
    like the eager loop: same sampled actions (same generator seeds), the same losses and weights after 5 updates
    within f32 tolerance (the capturable RMSprop keeps its step count on the device)."""
    from mfg_amd.factory import BatchedFactory
    from mfg_amd.marl import BatchedA2C
    res = {}
    for graph in (False, True):
        f = BatchedFactory('large8.yaml', 256, seed_base=5)
        torch.manual_seed(11)
        tr = BatchedA2C(f, n_steps=5, generator=torch.Generator(device='cuda').manual_seed(2), graph=graph)
        losses = [float(tr.train(1)) for _ in range(5)]
        assert tr.updates == 5 and (tr._graph is not None) == graph
        res[graph] = (losses, {n: p.detach().clone() for n, p in tr.net.named_parameters()},
                      tr.pobs.emb[0].clone())
        f.close()
    for a, b in zip(res[False][0], res[True][0]):
        assert abs(a - b) <= 1e-4 * max(1.0, abs(a)), (res[False][0], res[True][0])
    for n, p in res[False][1].items():
        assert torch.allclose(res[True][1][n], p, rtol=1e-4, atol=1e-5), n
    assert torch.allclose(res[True][2], res[False][2], rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
def test_batched_a2c_act_graph_replays_the_policy():
    """act_graph=True: every window slot's policy step is a captured HIP graph after two eager warm-ups; a replay
    computes the same recurrent states as the eager policy on the same inputs (the sampled actions draw from the
    graph's own Philox offsets), and training runs on."""
    from mfg_amd.factory import BatchedFactory
    from mfg_amd.marl import BatchedA2C
    f = BatchedFactory('large8.yaml', 256, seed_base=3)
    tr = BatchedA2C(f, n_steps=5, check_cap=True, act_graph=True)
    tr.train(4)
    assert sorted(tr._act_graphs) == list(range(5))
    tr._act_graphs[0].replay()
    ha_g, hc_g, sv_g, mx_g = tr.hs_a[0].clone(), tr.hs_c[0].clone(), tr.sv_a[:, 0].clone(), tr.mx[0].clone()
    tr._policy(0)
    assert torch.equal(ha_g, tr.hs_a[0]) and torch.equal(hc_g, tr.hs_c[0]) and torch.equal(sv_g, tr.sv_a[:, 0])
    assert torch.equal(mx_g, tr.mx[0])
    assert bool(torch.isfinite(tr.train(2)))
    assert int(tr.act.min()) >= 0 and int(tr.act.max()) < tr.n_actions
    f.close()


@pytest.mark.gpu
def test_a2c_loss_from_engine_projection_matches_gather():
    """The learner's obs_proj forward taken from the render's fused output gives the embedding_bag loss and
    gradients (f32 tolerance): every window slot was rendered with the current weights."""
    from mfg_amd.factory import BatchedFactory
    from mfg_amd.marl import BatchedA2C
    f = BatchedFactory('large8.yaml', 256, seed_base=2)
    tr = BatchedA2C(f, n_steps=5, generator=torch.Generator(device='cuda').manual_seed(1))
    tr.train(2)  # weights moved away from init; o_0 re-projected by the gather
    learn, tr.learn = tr.learn, (lambda: None)
    for _ in range(tr.T):
        tr.step()
    tr.learn = learn
    res = {}
    for mode in (True, False):
        tr.engine_emb = mode
        tr.net.zero_grad()
        loss = tr.loss()
        loss.backward()
        res[mode] = (float(loss), {n: p.grad.detach().clone() for n, p in tr.net.named_parameters() if p.grad is not None})
    assert abs(res[True][0] - res[False][0]) <= 1e-5 * max(1.0, abs(res[False][0]))
    for n, g in res[False][1].items():
        assert torch.allclose(res[True][1][n], g, rtol=1e-3, atol=1e-6), n
    f.close()


def test_windowed_gru_segments_match_the_step_loop():
    """One packed nn.GRU call over each row's episode segments == the step-by-step recurrence with the state
    zeroed at every restart (outputs and gradients, f32 tolerance)."""
    import torch
    from mfg_amd.marl import _Segments, _gru_cell
    torch.manual_seed(0)
    n, t, i, h = 37, 6, 20, 16
    gru = torch.nn.GRU(i, h, batch_first=True)
    x = torch.randn(n, t, i, requires_grad=True)
    h0 = torch.randn(n, h)
    starts = torch.rand(n, t) < 0.2
    starts[:, 0] = False
    starts[3] = True  # every entry restarts
    out = _Segments(starts, n, t, x.device).run(gru, x, h0)
    gi = torch.nn.functional.linear(x, gru.weight_ih_l0, gru.bias_ih_l0)
    hs, ref = h0, []
    for s in range(t):
        hs = hs * (~starts[:, s:s + 1]).float()
        hs = _gru_cell(gi[:, s], hs, gru)
        ref.append(hs)
    ref = torch.stack(ref, 1)
    assert torch.allclose(out, ref, atol=1e-5, rtol=1e-5)
    g1 = torch.autograd.grad(out.square().sum(), [x, gru.weight_hh_l0])
    g2 = torch.autograd.grad(ref.square().sum(), [x, gru.weight_hh_l0])
    for a, b in zip(g1, g2):
        assert torch.allclose(a, b, atol=1e-4, rtol=1e-4)


def test_fused_gru_window_matches_cells():
    """gru_window 'fused' (_GRUWindow: both GRUs, batched window GEMMs, hand-written backward) equals the
    per-step torch.gru_cell loop under autograd: outputs and every parameter gradient, with restarts."""
    torch.manual_seed(3)
    N, T = 5, 6
    nets = {m: RecurrentAC((2, 3, 3), 7, 12, 4, 8, 6, N, use_agent_embedding=False, gru_window=m)
            for m in ('fused', 'cells')}
    nets['cells'].load_state_dict(nets['fused'].state_dict())
    emb = torch.randn(N, T, 12)
    acts = torch.randint(-1, 7, (N, T))
    ha, hc = torch.randn(N, 1, 8), torch.randn(N, 1, 6)
    starts = torch.rand(N, T) < 0.25
    res = {}
    for m, net in nets.items():
        out = net.forward_emb(emb, acts, ha, hc, agent_ids=torch.arange(N), starts=starts)
        (out['logits'].square().sum() + out['critic'].sin().sum()).backward()
        res[m] = (out, {k: p.grad.clone() for k, p in net.named_parameters() if p.grad is not None})
    for k in ('logits', 'critic', 'hidden_actor', 'hidden_critic'):
        assert torch.allclose(res['fused'][0][k], res['cells'][0][k], rtol=1e-5, atol=1e-6), k
    assert res['fused'][1].keys() == res['cells'][1].keys()
    for k, g in res['cells'][1].items():
        assert torch.allclose(res['fused'][1][k], g, rtol=1e-4, atol=1e-6), (k, (res['fused'][1][k] - g).abs().max())


def test_split_k_weight_gradients_match_autograd(monkeypatch):
    """The learner's split-K layers (_tall_tn weight gradients: _Linear, _Embed with padding_idx, the GRU window)
    give nn.Linear / nn.Embedding / autograd's gradients on a window, forced to split at 64 rows."""
    import mfg_amd.marl as M
    torch.manual_seed(3)
    net = M.RecurrentAC(40, 5, 24, 8, 16, 16, 4, use_agent_embedding=False)
    n, t = 96, 6
    emb = torch.randn(n, t, 24)
    acts = torch.randint(-1, 5, (n, t))
    h0 = torch.zeros(n, 1, 16)
    starts = torch.rand(n, t) < 0.1
    res = {}
    for rows in (64, 1 << 30):
        monkeypatch.setattr(M, 'SPLIT_ROWS', rows)  # restored by pytest, also on failure
        net.zero_grad()
        out = net.forward_emb(emb, acts, h0, h0, starts=starts)
        (out['logits'].square().sum() + out['critic'].sum()).backward()
        res[rows] = {k: p.grad.clone() for k, p in net.named_parameters() if p.grad is not None}
    a, b = res[64], res[1 << 30]
    assert a.keys() == b.keys() and 'action_emb.weight' in a
    assert float(a['action_emb.weight'][0].abs().sum()) == 0.0
    for k in a:
        assert torch.allclose(a[k], b[k], rtol=1e-4, atol=1e-5), (k, (a[k] - b[k]).abs().max())
    # and the split path against plain autograd over nn modules (the 'cells' window, unsplit layers)
    net.gru_window = 'cells'
    net.zero_grad()
    out = net.forward_emb(emb, acts, h0, h0, starts=starts)
    (out['logits'].square().sum() + out['critic'].sum()).backward()
    for k, p in net.named_parameters():
        if p.grad is not None:
            assert torch.allclose(a[k], p.grad, rtol=1e-4, atol=1e-5), (k, (a[k] - p.grad).abs().max())


@pytest.mark.gpu
def test_gru_window_kernels_match_tensor_code(monkeypatch):
    """The learner's GRU window on the GPU through libmfg_hip.so's fused step kernels (mfg_gru_fwd_step /
    mfg_gru_bwd_step, include/mfg_learn.h) against the same window in tensor code, forward and every gradient
    (fp32; the kernels follow the tensor code's formulas, libm exp/tanh may round differently)."""
    from conftest import gpu_available
    if not gpu_available():
        pytest.skip('no GPU')
    import mfg_amd.marl as M
    torch.manual_seed(5)
    net = M.RecurrentAC(40, 5, 24, 8, 16, 16, 4, use_agent_embedding=False).cuda()
    n, t = 3000, 6
    emb = torch.randn(n, t, 24, device='cuda')
    acts = torch.randint(-1, 5, (n, t), device='cuda')
    h0 = torch.randn(n, 1, 16, device='cuda')
    starts = torch.rand(n, t, device='cuda') < 0.1
    res = {}
    orig = M._use_gru_kernels
    for kern in (True, False):
        monkeypatch.setattr(M, '_use_gru_kernels', orig if kern else (lambda x: False))  # restored on failure too
        net.zero_grad()
        out = net.forward_emb(emb, acts, h0, h0, starts=starts)
        (out['logits'].square().sum() + out['critic'].sum()).backward()
        res[kern] = ({k: out[k].detach().clone() for k in ('logits', 'critic', 'hidden_actor', 'hidden_critic')},
                     {k: p.grad.clone() for k, p in net.named_parameters() if p.grad is not None})
    for k in res[True][0]:
        assert torch.allclose(res[True][0][k], res[False][0][k], rtol=1e-5, atol=1e-6), k
    for k in res[False][1]:
        a, b = res[True][1][k], res[False][1][k]
        assert torch.allclose(a, b, rtol=1e-4, atol=1e-5), (k, (a - b).abs().max())


@pytest.mark.gpu
def test_batched_a2c_saved_window_matches_recompute():
    """reuse_acting (the default): the learner takes the mix's and the GRUs' forward from the acting steps (stored
    activations, entry-major) and evaluates the entry-T bootstrap critic by one no-grad step; loss and every
    gradient equal the full-window recompute (the reference learner's order) within f32 tolerance."""
    from mfg_amd.factory import BatchedFactory
    from mfg_amd.marl import BatchedA2C
    f = BatchedFactory('large8.yaml', 256, seed_base=4)
    tr = BatchedA2C(f, n_steps=5, generator=torch.Generator(device='cuda').manual_seed(3))
    assert tr.reuse
    tr.train(2)  # weights moved away from init, episode restarts inside windows possible
    learn, tr.learn = tr.learn, (lambda: None)
    for _ in range(tr.T):
        tr.step()
    tr.learn = learn
    res = {}
    for name, fn in (('saved', tr._loss_saved), ('recompute', tr._loss_recompute)):
        tr.net.zero_grad()
        loss = fn()
        loss.backward()
        res[name] = (float(loss), {n: p.grad.detach().clone() for n, p in tr.net.named_parameters()
                                   if p.grad is not None})
    a, b = res['saved'][0], res['recompute'][0]
    assert abs(a - b) <= 1e-5 * max(1.0, abs(b)), (a, b)
    assert set(res['saved'][1]) == set(res['recompute'][1])
    for n, g in res['recompute'][1].items():
        assert torch.allclose(res['saved'][1][n], g, rtol=1e-3, atol=1e-6), (n, (res['saved'][1][n] - g).abs().max())
    f.close()


def _rand_packed(m, cap, k, gen, fill=0.7):
    """Random packed rows: distinct indices per row, nonzero values, ~fill of the cap slots used (zeros after)."""
    idx = torch.zeros((m, cap), dtype=torch.int64)
    val = torch.zeros((m, cap), dtype=torch.float32)
    cnt = torch.randint(0, cap + 1, (m,), generator=gen)
    cnt = torch.where(torch.rand(m, generator=gen) < fill, cnt, torch.full_like(cnt, cap))
    perm = torch.rand((m, k), generator=gen).argsort(1)[:, :cap]
    used = torch.arange(cap)[None, :] < cnt[:, None]
    idx[used] = perm[used]
    val[used] = torch.rand(int(used.sum()), generator=gen) * 2 + 0.25
    return idx, val


@pytest.mark.gpu
@pytest.mark.parametrize('m,cap,k,e', [(5000, 32, 343, 96), (3000, 70, 1000, 96), (777, 8, 50, 20), (600, 16, 5000, 24)])
def test_packed_grads_match_dense(m, cap, k, e):
    """The learner's obs_proj gradients from packed rows (mfg_packed_densify, bit-exact dense rows, then the split-K
    GEMM; C3's k = 343, a wide k = 1000, cap 70 past one wave) against the dense rows' f64 GEMM and column sum."""
    import mfg_amd.marl as M
    gen = torch.Generator().manual_seed(m)
    idx, val = _rand_packed(m, cap, k, gen)
    g = torch.randn((m, e), generator=gen)
    d = torch.zeros((m, k), dtype=torch.float64)
    d.scatter_add_(1, idx, val.double())
    iu, vc = idx.to(torch.uint16).cuda(), val.cuda()
    if k <= M._DENSIFY_MAX_K:
        dd = torch.full((m, k + 3), -1.0, device='cuda')  # row stride k + 3: the pad columns stay untouched
        assert M._gru_lib().mfg_packed_densify(iu.data_ptr(), vc.data_ptr(), m, cap, k, dd.data_ptr(), k + 3,
                                               torch.cuda.current_stream().cuda_stream) == 0
        assert torch.equal(dd[:, :k].cpu(), d.float()) and bool((dd[:, k:] == -1).all())
    else:  # past the kernel's bound: refused, and _packed_grads takes the scatter_add rows instead
        dd = torch.empty((m, k), device='cuda')
        assert M._gru_lib().mfg_packed_densify(iu.data_ptr(), vc.data_ptr(), m, cap, k, dd.data_ptr(), k,
                                               torch.cuda.current_stream().cuda_stream) == -1
    ref_w, ref_b = (d.t() @ g.double()).t(), g.double().sum(0)
    gw, gb = M._packed_grads(iu, vc, g.cuda(), k)
    assert gw.shape == (e, k) and gb.shape == (e,)
    assert torch.allclose(gw.double().cpu(), ref_w, rtol=1e-4, atol=1e-4), (gw.double().cpu() - ref_w).abs().max()
    assert torch.allclose(gb.double().cpu(), ref_b, rtol=1e-4, atol=1e-4)


@pytest.mark.gpu
def test_packed_project_kernel_matches_dense():
    """mfg_packed_project (the learner's slot-0 re-projection) against bias + dense rows @ W^T in f64."""
    import mfg_amd.marl as M
    gen = torch.Generator().manual_seed(9)
    m, cap, k, e = 4000, 70, 343, 96
    idx, val = _rand_packed(m, cap, k, gen)
    w, b = torch.randn((e, k), generator=gen), torch.randn(e, generator=gen)
    d = torch.zeros((m, k), dtype=torch.float64)
    d.scatter_add_(1, idx, val.double())
    ref = d @ w.double().t() + b.double()
    out = torch.empty((m, e), device='cuda')
    L = M._gru_lib()
    iu, vc, wt, bc = idx.to(torch.uint16).cuda(), val.cuda(), w.t().contiguous().cuda(), b.cuda()
    assert L.mfg_packed_project(iu.data_ptr(), vc.data_ptr(), m, cap, wt.data_ptr(), bc.data_ptr(), e, k,
                                out.data_ptr(), e, torch.cuda.current_stream().cuda_stream) == 0
    assert torch.allclose(out.double().cpu(), ref, rtol=1e-5, atol=1e-4)


@pytest.mark.gpu
def test_sample_categorical_kernel_distribution():
    """mfg_sample_categorical: inversion sampling at caller-drawn uniforms; exact picks at chosen uniforms and the
    empirical frequencies of 2M draws within 0.003 of softmax(logits)."""
    import mfg_amd.marl as M
    L = M._gru_lib()
    st = torch.cuda.current_stream().cuda_stream
    logits = torch.tensor([0.5, -1.0, 2.0, 0.0, 1.0], device='cuda')
    p = torch.softmax(logits.double(), 0).cpu()
    cdf = p.cumsum(0)
    # exact picks: u just below / above each CDF step
    us = torch.cat([cdf[:-1] - 1e-4, cdf[:-1] + 1e-4, torch.tensor([0.0, 0.999999])]).float().cuda()
    n = us.numel()
    lg = logits.repeat(n, 1).contiguous()
    out = torch.empty(n, dtype=torch.int32, device='cuda')
    assert L.mfg_sample_categorical(lg.data_ptr(), 5, 5, us.data_ptr(), n, out.data_ptr(), st) == 0
    exp = torch.searchsorted(cdf, us.double().cpu(), right=True).clamp(max=4)
    assert torch.equal(out.cpu().long(), exp)
    n = 2_000_000
    lg = logits.repeat(n, 1).contiguous()
    u = torch.rand(n, device='cuda')
    out = torch.empty(n, dtype=torch.int32, device='cuda')
    assert L.mfg_sample_categorical(lg.data_ptr(), 5, 5, u.data_ptr(), n, out.data_ptr(), st) == 0
    freq = torch.bincount(out.long(), minlength=5).double().cpu() / n
    assert float((freq - p).abs().max()) < 3e-3, (freq, p)
    # non-finite logits: no distribution, the row is marked -1 (BatchedA2C.learn raises on it)
    bad = torch.tensor([[0.0, float('nan'), 1.0], [float('inf'), 0.0, 0.0], [0.0, 1.0, 2.0]], device='cuda')
    u3 = torch.full((3,), 0.5, device='cuda')
    o3 = torch.empty(3, dtype=torch.int32, device='cuda')
    assert L.mfg_sample_categorical(bad.data_ptr(), 3, 3, u3.data_ptr(), 3, o3.data_ptr(), st) == 0
    assert o3.cpu().tolist()[:2] == [-1, -1] and 0 <= int(o3[2]) < 3


def test_saved_mix_backward_matches_autograd():
    """_MixSaved (the learner's mix from the acting steps' stored activations): forward == net.mix on the same
    inputs and every gradient (obs_emb, both layers, the action embedding with its padding row) == autograd's."""
    import mfg_amd.marl as M
    torch.manual_seed(0)
    net = M.RecurrentAC(40, 5, 24, 8, 16, 16, 4, use_agent_embedding=False)
    rows = 300
    emb = torch.randn(rows, 24, requires_grad=True)
    a = torch.randint(-1, 5, (rows,))
    params = [emb, net.mix[1].weight, net.mix[1].bias, net.mix[3].weight, net.mix[3].bias, net.action_emb.weight]
    x = torch.cat([emb, net.action_emb(a + 1)], 1)
    ref = net.mix(x)
    g = torch.randn_like(ref)
    gr = torch.autograd.grad(ref, params, g)
    with torch.no_grad():
        ax = torch.tanh(x)
        h1 = torch.tanh(net.mix[1](ax))
        mx = net.mix[3](h1)
    out = M._MixSaved.apply(emb, *params[1:], (ax, h1, mx, a, net.action_emb.padding_idx))
    gs = torch.autograd.grad(out, params, g)
    assert torch.allclose(out, ref, atol=1e-6)
    for p, q in zip(gs, gr):
        assert torch.allclose(p, q, rtol=1e-5, atol=1e-6), (p - q).abs().max()

#!/usr/bin/env python3
"""GPU debugging aid: step B envs of a config on the HIP engine beside the C oracle (Philox actions) and
print the first divergence with the engine's event rows and record header. usage: dbg_cfg.py CFG [B] [STEPS]"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT / 'marl-factory-grid_amd'), str(ROOT / 'oracle'), str(ROOT / 'tests')]
import torch  # noqa: E402
import oracle as O  # noqa: E402
from philox import synthetic_actions  # noqa: E402
from mfg_amd.spec import compile_spec  # noqa: E402
from mfg_amd.engine import Engine, RecordView, events_from_rows, EV_MISC, HDR  # noqa: E402

cfg = sys.argv[1]
B = int(sys.argv[2]) if len(sys.argv) > 2 else 2
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 50
spec = compile_spec(cfg)
eng = Engine(spec, B)
print('layout', {k: eng.layout[k] for k in ('size', 'lds_full', 'xchg_ordered')})
A, dev, nl = spec.n_agents, eng.device, spec.n_layers
obs = torch.zeros(eng.obs_shape(), dtype=torch.float64, device=dev)
base, pseed = 1000, 7
eng.reset(obs=obs, init=True, seed_base=base)
envs = [O.OracleEnv(spec, base + i) for i in range(B)]
for e in envs:
    e.reset()
rew = torch.zeros((1, B, A), dtype=torch.float64, device=dev)
done = torch.zeros((1, B), dtype=torch.uint8, device=dev)
ev_a = torch.zeros((1, B, A), dtype=torch.uint8, device=dev)
ev_w = torch.zeros((1, B, A), dtype=torch.uint8, device=dev)
ev_m = torch.zeros((1, B, EV_MISC), dtype=torch.int32, device=dev)
for t in range(steps):
    eng.step(1, actions=None, philox_seed=pseed, step_base=t, reward=rew, done=done, obs=obs, ev_act=ev_a,
             ev_watch=ev_w, ev_misc=ev_m, auto_reset=False)
    acts = synthetic_actions(pseed, np.arange(B), t, spec.n_actions)
    st = eng.export_state().cpu().numpy()
    bad = False
    for i, env in enumerate(envs):
        r_ref, d_ref, ev_ref = env.step(acts[i])
        rw, dn = rew[0, i].cpu().numpy(), bool(done[0, i].item())
        ev = events_from_rows(ev_a[0, i].cpu().numpy(), ev_w[0, i].cpu().numpy(), ev_m[0, i].cpu().numpy())
        rv = RecordView(st[i], eng.layout, spec)
        msg = []
        if list(rw) != list(r_ref):
            msg.append(f'reward idx {[a for a in range(A) if rw[a] != r_ref[a]][:8]}')
        if dn != d_ref:
            msg.append(f'done {dn} vs {d_ref}')
        if list(ev['act'][:A]) != list(ev_ref.act[:A]):
            msg.append('act events')
        if list(ev['watch'][:A]) != list(ev_ref.watch[:A]):
            msg.append('watch events')
        o = obs[i].cpu().numpy()
        ro = env.obs_list()
        for a in range(A):
            if not (o[a, :nl[a]] == ro[a]).all():
                dif = np.argwhere(o[a, :nl[a]] != ro[a])
                msg.append(f'obs agent {a}: {len(dif)} diffs {[(tuple(x), o[a][tuple(x)], ro[a][tuple(x)]) for x in dif[:4]]}')
                break
        if msg:
            print(f't{t} env{i}:', '; '.join(msg))
            print('  engine ev', {k: v for k, v in ev.items() if k not in ('act', 'watch')})
            print('  oracle ev', {k: getattr(ev_ref, k) for k in dir(ev_ref) if not k.startswith('_') and k not in ('act', 'watch')})
            h = st[i][eng.layout['o_hdr']:eng.layout['o_hdr'] + 4 * 40].view(np.int32)
            print('  hdr', {k: int(h[v]) for k, v in HDR.items()})
            L = eng.layout
            print('  layout', {k: L[k] for k in ('size', 'dirt_cap', 'lds_full', 'lds_logic', 'lds_obs', 'lds_replay',
                                                 'bfs_off', 'bfs_bytes', 'max_pairs', 'scratch_bytes', 'o_grank')})
            if L['bfs_bytes']:
                g = st[i][L['o_grank']:L['o_grank'] + 2 * len(spec.floor_cells)].view(np.uint16)
                print('  grank perm ok', sorted(g.tolist()) == list(range(len(g))), 'nonzero', int((g > 0).sum()))
                ms = st[i][L['o_mstate']:L['o_mstate'] + 4 * 13 * 4].view(np.int32).reshape(4, 13)
                print('  mstate', ms.tolist())
                mw = st[i][L['o_maints']:L['o_maints'] + 16].view(np.int32)
                print('  maints', [(int(w) & 0xFFFF, hex(int(w) >> 16)) for w in mw])
            bad = True
    if bad:
        break
    if t % 10 == 0:
        print('t', t, 'ok', flush=True)
eng.close()

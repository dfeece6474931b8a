#!/usr/bin/env python3
"""Device kernels of one A2C learner update (loss forward + backward + clip/RMSprop, BatchedA2C, C3 large8), torch
profiler, kernel rows only (no aten:: op rows), per update. usage: python tools/prof_a2c_learn.py [--batch 8192]
[--recompute] (the full-window recompute learner instead of the stored acting pass)"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / 'marl-factory-grid_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=8192)
    ap.add_argument('--updates', type=int, default=3)
    ap.add_argument('--recompute', action='store_true')
    ap.add_argument('--split-rows', type=int, default=0, help='marl.SPLIT_ROWS (rows per split-K GEMM batch)')
    args = ap.parse_args()
    import torch
    from torch.profiler import profile, ProfilerActivity
    from mfg_amd.factory import BatchedFactory
    from mfg_amd.marl import BatchedA2C
    import mfg_amd.marl as M
    if args.split_rows:
        M.SPLIT_ROWS = args.split_rows
    f = BatchedFactory('large8.yaml', args.batch, seed_base=0)
    tr = BatchedA2C(f, n_steps=5, check_cap=True)
    if args.recompute:
        tr.loss = tr._loss_recompute
    tr.train(2)
    learn, tr.learn = tr.learn, (lambda: None)
    for _ in range(tr.T):
        tr.step()
    tr.learn = learn

    def upd():
        with torch.enable_grad():
            loss = tr.loss()
            tr.opt.zero_grad(set_to_none=True)
            loss.backward()
            torch.nn.utils.clip_grad_norm_(tr.net.parameters(), 0.5)
            tr.opt.step()
    upd()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        for _ in range(args.updates):
            upd()
        torch.cuda.synchronize()
    rows = []
    for e in prof.key_averages():
        if e.self_device_time_total <= 0 or e.key.startswith('aten::') or e.key.startswith('autograd::'):
            continue
        rows.append((e.self_device_time_total / args.updates, e.count / args.updates, e.key))
    rows.sort(reverse=True)
    tot = sum(r[0] for r in rows)
    print(f'learner update ({"recompute" if args.recompute else "saved acting pass"}), B={args.batch}, '
          f'SPLIT_ROWS {M.SPLIT_ROWS}: '
          f'{tot / 1e3:.3f} ms device kernels per update')
    for us, n, k in rows[:40]:
        print(f'{us / 1e3:8.3f} ms {n:6.1f}x  {k[:120]}')
    f.close()


if __name__ == '__main__':
    main()

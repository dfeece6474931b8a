#!/usr/bin/env python3
"""Kernels of the A2C acting step (policy forward on the fused projection, sampling, mfg_step, bookkeeping), torch
profiler over 10 steps without the update. usage: python tools/prof_a2c_act.py [--batch 8192]"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / 'marl-factory-grid_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=8192)
    args = ap.parse_args()
    import torch
    from torch.profiler import profile, ProfilerActivity
    from mfg_amd.factory import BatchedFactory
    from mfg_amd.marl import BatchedA2C
    f = BatchedFactory('large8.yaml', args.batch, seed_base=0)
    tr = BatchedA2C(f, n_steps=5, check_cap=True)
    tr.train(2)
    tr.learn = lambda: setattr(tr, 't', 0)
    for _ in range(5):
        tr.step()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        for _ in range(10):
            tr.step()
        torch.cuda.synchronize()
    ka = prof.key_averages()
    print(ka.table(sort_by='self_device_time_total', row_limit=40, max_name_column_width=70))
    f.close()


if __name__ == '__main__':
    main()

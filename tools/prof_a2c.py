#!/usr/bin/env python3
"""Where the on-GPU A2C loop's time goes: wall time per update against the GPU kernel time inside it
(torch.profiler), and the top kernels. usage: python tools/prof_a2c.py [--batch 8192] [--updates 3]"""
import argparse
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / 'marl-factory-grid_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='large8.yaml')
    ap.add_argument('--batch', type=int, default=8192)
    ap.add_argument('--updates', type=int, default=3)
    ap.add_argument('--blas', default=None, help="torch.backends.cuda.preferred_blas_library ('cublas' = rocBLAS, "
                                                 "'cublaslt' = hipBLASLt)")
    ap.add_argument('--gather', action='store_true', help='learner obs_proj forward by embedding_bag')
    args = ap.parse_args()
    import torch
    if args.blas:
        torch.backends.cuda.preferred_blas_library(args.blas)
    from torch.profiler import profile, ProfilerActivity
    from mfg_amd.factory import BatchedFactory
    from mfg_amd.marl import BatchedA2C
    f = BatchedFactory(args.config, args.batch, seed_base=0)
    tr = BatchedA2C(f, n_steps=5, check_cap=True, engine_emb=not args.gather)
    tr.train(3)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.train(args.updates)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / args.updates * 1e3
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        tr.train(args.updates)
        torch.cuda.synchronize()
    ka = prof.key_averages()
    dev_us = sum(e.self_device_time_total for e in ka) / args.updates
    n_k = sum(e.count for e in ka if e.self_device_time_total > 0) / args.updates
    print(f'wall {wall:.2f} ms/update, device kernels {dev_us / 1e3:.2f} ms/update, {n_k:.0f} device ops/update')
    print(ka.table(sort_by='self_device_time_total', row_limit=25, max_name_column_width=60))
    f.close()


if __name__ == '__main__':
    main()

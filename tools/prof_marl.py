#!/usr/bin/env python3
"""torch.profiler breakdown of the on-GPU A2C loop (tools/bench_marl.py's workload): top device ops."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / 'marl-factory-grid_amd'))


def main():
    import torch
    from torch.profiler import profile, ProfilerActivity
    from mfg_amd.factory import BatchedFactory
    from mfg_amd.marl import BatchedA2C
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    f = BatchedFactory('large8.yaml', B, seed_base=0)
    tr = BatchedA2C(f, n_steps=5, check_cap=True)
    tr.train(2)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
        tr.train(3)
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by='cuda_time_total', row_limit=25))
    print(prof.key_averages().table(sort_by='cpu_time_total', row_limit=15))


if __name__ == '__main__':
    main()

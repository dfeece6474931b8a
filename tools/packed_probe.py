#!/usr/bin/env python3
"""k_obs time per launch by obs mode (C3, B=65536, K=8): dense f32, packed entries only, fused projection
only, both. Timing probe for the packed-obs kernel."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / 'marl-factory-grid_amd'))


def main():
    import torch
    from mfg_amd.spec import compile_spec
    from mfg_amd.engine import Engine, PackedObs
    spec = compile_spec('large8.yaml')
    B, F = 65536, 8
    e = Engine(spec, B, device=0)
    kdim = e.lmax * e.obs_hw[0] * e.obs_hw[1]
    w = torch.randn(96, kdim, device='cuda') * 0.05
    e.reset(obs=None, init=True)
    modes = {'dense_f32': torch.zeros((F,) + e.obs_shape(), dtype=torch.float32, device='cuda'),
             'entries': PackedObs(e, K=F, cap=32),
             'emb_only': PackedObs(e, K=F, cap=32, weight=w, entries=False),
             'entries+emb': PackedObs(e, K=F, cap=32, weight=w)}
    for name, o in modes.items():
        e.step(F, philox_seed=1, step_base=0, obs=o)
        e.profile(True)
        e.profile_read()
        for c in range(10):
            e.step(F, philox_seed=1, step_base=8 * (c + 1), obs=o)
        p = e.profile_read()
        e.profile(False)
        print(name, {k: round(ms / n, 4) for k, (ms, n) in p.items() if n})


if __name__ == '__main__':
    main()

#!/usr/bin/env python3
"""Timing probe: C3 (large8, B=65536, K=8, dense f32 obs, auto_reset off) calls per second with the call's
k_replay serialised (default) or overlapped with the next call on a second stream (MFG_ABLATE_OVERLAP=1, a
measurement switch whose results are not exact). Prints one line per mode; each mode runs in its own
process because the switch is read once per process."""
import os
import subprocess
import sys
import time
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / 'marl-factory-grid_amd'))


def run(calls=30):
    import torch
    from mfg_amd.spec import compile_spec
    from mfg_amd.engine import Engine
    spec = compile_spec('large8.yaml')
    B, F = 65536, 8
    e = Engine(spec, B, device=0)
    obs = torch.zeros((F,) + e.obs_shape(), dtype=torch.float32, device='cuda')
    rew = torch.zeros((F, B, e.A), dtype=torch.float64, device='cuda')
    done = torch.zeros((F, B), dtype=torch.uint8, device='cuda')
    e.reset(obs=None, init=True)
    for c in range(5):
        e.step(F, philox_seed=1, step_base=8 * c, obs=obs, reward=rew, done=done, auto_reset=False)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for c in range(calls):
        e.step(F, philox_seed=1, step_base=8 * (c + 5), obs=obs, reward=rew, done=done, auto_reset=False)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t) * 1e3 / calls
    print(f"overlap={os.environ.get('MFG_ABLATE_OVERLAP', '0')} ms_per_call={ms:.3f} "
          f"env_steps_per_s={B * F / ms * 1e3 / 1e6:.2f}M", flush=True)


if __name__ == '__main__':
    if len(sys.argv) > 1 and sys.argv[1] == 'child':
        run()
    else:
        for ov in ('0', '1', '0', '1'):
            env = dict(os.environ, MFG_ABLATE_OVERLAP=ov)
            subprocess.run([sys.executable, __file__, 'child'], env=env, check=True, timeout=300)

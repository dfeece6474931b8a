#!/usr/bin/env python3
"""Timing probe: the C3 bench workload (65,536 envs) as S engines of 65,536/S envs on S HIP streams in one
process, against one engine on one stream. Same trajectories (env_base offsets), different overlap."""
import sys, time
from pathlib import Path
ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / 'marl-factory-grid_amd'))


def main():
    import torch
    from mfg_amd.spec import compile_spec
    from mfg_amd.engine import Engine
    spec = compile_spec('large8.yaml')
    B, F, steps, warm = 65536, 8, 800, 600
    for S in [int(x) for x in (sys.argv[1:] or ['1', '2', '4'])]:
        b = B // S
        engs, bufs, streams = [], [], []
        for i in range(S):
            e = Engine(spec, b, device=0)
            obs = torch.zeros((F,) + e.obs_shape(), dtype=torch.float32, device='cuda')
            rew = torch.zeros((F, b, spec.n_agents), dtype=torch.float64, device='cuda')
            done = torch.zeros((F, b), dtype=torch.uint8, device='cuda')
            e.reset(obs=obs[0], init=True, seed_base=i * b)
            engs.append(e); bufs.append((obs, rew, done)); streams.append(torch.cuda.Stream())
        torch.cuda.synchronize()

        def run(n, t0):
            for k in range(0, n, F):
                for i, e in enumerate(engs):
                    with torch.cuda.stream(streams[i]):
                        obs, rew, done = bufs[i]
                        e.step(F, philox_seed=12345, env_base=i * b, step_base=t0 + k, reward=rew, done=done, obs=obs)
        run(warm, 0)
        torch.cuda.synchronize()
        t = time.perf_counter()
        run(steps, warm)
        torch.cuda.synchronize()
        el = time.perf_counter() - t
        print(f'S={S}: {B * steps / el / 1e6:.2f}M env-steps/s, {el / steps * 1e3:.4f} ms/step', flush=True)
        for e in engs:
            e.close()
        del engs, bufs
        torch.cuda.empty_cache()


if __name__ == '__main__':
    main()

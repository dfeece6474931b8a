"""One rank of tests/test_gpu_ranks.py: a fresh process (started by the test with RANK / WORLD_SIZE / MASTER_*
set, like torch.distributed.run) that joins a gloo process group, steps its own env shard with the HIP engine
on GPU 0 (several ranks share the one GPU of the test box) and gathers its outputs to rank 0, which writes them
to OUT. Nothing here touches the GPU before the process group is up."""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT / 'marl-factory-grid_amd', ROOT / 'tests'):
    sys.path.insert(0, str(p))


def main():
    cfg, per_rank, steps, K, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
    import numpy as np
    import torch
    import torch.distributed as dist
    from mfg_amd.engine import EV_MISC, Engine
    from mfg_amd.shard import allreduce_metrics, env_range
    from mfg_amd.spec import compile_spec
    rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
    dist.init_process_group('gloo')
    assert dist.get_world_size() == world
    torch.cuda.set_device(0)
    spec = compile_spec(cfg)
    first, count = env_range(rank, world, per_rank)
    eng = Engine(spec, count, device=0)
    dev, A = eng.device, spec.n_agents
    obs = torch.zeros((K,) + eng.obs_shape(), dtype=torch.float64, device=dev)
    rew = torch.zeros((K, count, A), dtype=torch.float64, device=dev)
    done = torch.zeros((K, count), dtype=torch.uint8, device=dev)
    ev = [torch.zeros((K, count, A), dtype=torch.uint8, device=dev) for _ in range(2)]
    evm = torch.zeros((K, count, EV_MISC), dtype=torch.int32, device=dev)
    eng.reset(obs=obs[0], init=True, seed_base=first)
    R, D = [], []
    for t0 in range(0, steps, K):
        eng.step(K, actions=None, philox_seed=31, env_base=first, step_base=t0, reward=rew, done=done, obs=obs,
                 ev_act=ev[0], ev_watch=ev[1], ev_misc=evm, auto_reset=True)
        R.append(rew.cpu().clone())
        D.append(done.cpu().clone())
    # obs of the last call only (every step's rewards / done, the final state records incl. MT and floor order)
    mine = {'reward': torch.cat(R), 'done': torch.cat(D), 'obs': obs.cpu().clone(), 'state': eng.export_state().cpu()}
    eps = allreduce_metrics(torch.tensor([float(mine['done'].sum())], dtype=torch.float64))
    gathered = {}
    for k, v in mine.items():  # gather along the env axis (axis 1 for per-step rows, 0 for the state records)
        parts = [torch.zeros_like(v) for _ in range(world)]
        dist.all_gather(parts, v.contiguous())
        gathered[k] = torch.cat(parts, dim=0 if k == 'state' else 1).numpy()
    if rank == 0:
        np.savez(out, episodes=eps.numpy(), **gathered)
    dist.barrier()
    eng.close()
    dist.destroy_process_group()


if __name__ == '__main__':
    main()

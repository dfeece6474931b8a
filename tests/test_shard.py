"""Multi-process (gloo, world_size 2) coverage of the sharded path on CPU: each rank owns a contiguous
env range keyed by global env index, steps its envs independently (C oracle as the per-env stepper —
on the GPU box the HIP engine takes this place), and only a metrics vector is all-reduced. The union of
the ranks' results must equal a single-process run over all envs."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from mfg_amd.shard import env_range, split_global

STEPS, PER_RANK, SEED = 60, 3, 77


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rollout(first, count):
    import oracle as O
    from philox import synthetic_actions
    from mfg_amd.spec import compile_spec
    spec = compile_spec('rooms4.yaml')
    out = []
    for env in range(first, first + count):
        e = O.OracleEnv(spec, 500 + env)
        e.reset()
        rs, eps = [], 0
        for t in range(STEPS):
            r, d, _ = e.step(synthetic_actions(SEED, [env], t, spec.n_actions)[0])
            rs.append(list(r))
            if d:
                eps += 1
                e.reset()
        out.append((env, np.asarray(rs), eps))
    return out


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    first, count = env_range(rank, world, PER_RANK)
    res = _rollout(first, count)
    from mfg_amd.shard import allreduce_metrics
    m = allreduce_metrics(torch.tensor([float(sum(r.sum() for _, r, _ in res)), float(len(res) * STEPS)],
                                       dtype=torch.float64))
    q.put((rank, [(e, r.tolist(), n) for e, r, n in res], m.tolist()))
    dist.barrier()
    dist.destroy_process_group()


def test_env_ranges():
    assert [env_range(r, 4, 10) for r in range(4)] == [(0, 10), (10, 10), (20, 10), (30, 10)]
    parts = [split_global(r, 3, 10) for r in range(3)]
    assert parts == [(0, 4), (4, 3), (7, 3)] and sum(c for _, c in parts) == 10
    with pytest.raises(ValueError):
        env_range(2, 2, 5)


def test_gloo_world2_matches_single_process():
    world = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = {e: (r, n) for e, r, n in _rollout(0, world * PER_RANK)}
    total = 0.0
    for rank, res, metrics in got:
        for e, r, n in res:
            assert np.array_equal(np.asarray(r), ref[e][0]) and n == ref[e][1], f'env {e} on rank {rank}'
            total += float(np.asarray(r).sum())
    for _, _, metrics in got:
        assert metrics[1] == world * PER_RANK * STEPS
        assert abs(metrics[0] - total) < 1e-9


ROOT = __import__('pathlib').Path(__file__).resolve().parent.parent


def _bench(*args, timeout=240):
    import subprocess
    import sys
    env = dict(os.environ, MASTER_ADDR='127.0.0.1')
    env.pop('WORLD_SIZE', None)
    return subprocess.run([sys.executable, str(ROOT / 'bench.py'), *args], capture_output=True, text=True,
                          timeout=timeout, env=env, cwd=str(ROOT))


def test_bench_spawns_ranks_and_collects_rank0_line():
    """`bench.py --gpus 2` (the driver's SCALE command form) starts 2 rank processes itself, joins them in one
    process group (gloo rehearsal: --dry-run), takes the MAX over ranks and prints exactly one JSON line."""
    import json
    p = _bench('--gpus', '2', '--dry-run', '--steps', '5', '--batch', '8')
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d['n_gpus'] == 2 and d['backend'] == 'gloo' and d['n_ranks_gloo'] == 2 and d['dry_run']
    assert d['env_ranges'] == [[0, 8], [8, 8]]
    assert d['metrics_allreduce'] == 2 * 8 * 5
    assert 'launcher' in d


def test_bench_refuses_more_gpus_than_visible():
    import torch
    visible = torch.cuda.device_count()
    n = max(2, visible + 1)
    p = _bench('--gpus', str(n), '--steps', '2', '--warmup', '0', '--no-cpu-baseline')
    assert p.returncode == 2
    assert f'{n} GPUs requested, {visible} visible' in p.stderr
    assert not [ln for ln in p.stdout.splitlines() if ln.startswith('{')]


def test_bench_under_launcher_world1_joins_a_group():
    """Under torch.distributed.run with one process (the driver's N = 1 SCALE form) the rank joins a real process
    group of size 1 (gloo in this CPU rehearsal; nccl on the GPU, tests/test_gpu_ranks.py) instead of skipping it."""
    import json
    import socket
    import subprocess
    import sys
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ)
    env.pop('WORLD_SIZE', None)
    p = subprocess.run([sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '1',
                        '--master-addr', '127.0.0.1', '--master-port', str(port), str(ROOT / 'bench.py'), '--gpus', '1',
                        '--dry-run', '--steps', '3', '--batch', '8'], capture_output=True, text=True, timeout=300,
                       env=env, cwd=str(ROOT))
    assert p.returncode == 0, p.stderr[-2000:]
    d = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith('{')][-1])
    assert d['backend'] == 'gloo' and d['n_ranks_gloo'] == 1 and d['n_gpus'] == 1
    assert d['metrics_allreduce'] == 8 * 3

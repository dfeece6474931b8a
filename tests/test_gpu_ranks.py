"""The multi-rank path the driver's SCALE run takes, exercised on the one GPU of the test box (VERDICT r3 item
2): fresh rank processes (RANK / WORLD_SIZE / MASTER_* as torch.distributed.run sets them) each own a contiguous
global env range, step it with their own HIP engine, and gather over gloo; the union must equal one engine over
all envs bit-exactly (every step's rewards and done, the last call's obs, the full state records incl.
MT19937 and floor order); large8 runs across the episode-500 reset. A second test
runs bench.py --gpus 2 as its own launcher (launch_ranks) with both ranks sharing GPU 0."""
import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

from conftest import gpu_available

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _child_env(rank, world, port):
    env = dict(os.environ, RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR='127.0.0.1',
               MASTER_PORT=str(port))
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
    return env


@pytest.mark.timeout(600)
@pytest.mark.parametrize('cfg,per_rank,steps', [('large8.yaml', 64, 520), ('rooms4.yaml', 128, 96)])
def test_two_rank_processes_equal_one_engine(tmp_path, cfg, per_rank, steps):
    if not gpu_available():
        pytest.skip('no GPU')
    world, K = 2, 8
    out = tmp_path / 'ranks.npz'
    port = _free_port()
    procs = [subprocess.Popen([sys.executable, '-u', str(ROOT / 'tests' / 'shard_rank_worker.py'), cfg,
                               str(per_rank), str(steps), str(K), str(out)], env=_child_env(r, world, port))
             for r in range(world)]
    try:
        codes = [p.wait(timeout=500) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert codes == [0, 0], codes
    got = np.load(out)
    import torch
    from mfg_amd.engine import EV_MISC, Engine
    from mfg_amd.spec import compile_spec
    spec = compile_spec(cfg)
    B, A = world * per_rank, spec.n_agents
    eng = Engine(spec, B, device=0)
    dev = eng.device
    obs = torch.zeros((K,) + eng.obs_shape(), dtype=torch.float64, device=dev)
    rew = torch.zeros((K, B, A), dtype=torch.float64, device=dev)
    done = torch.zeros((K, B), dtype=torch.uint8, device=dev)
    ev = [torch.zeros((K, B, A), dtype=torch.uint8, device=dev) for _ in range(2)]
    evm = torch.zeros((K, B, EV_MISC), dtype=torch.int32, device=dev)
    eng.reset(obs=obs[0], init=True, seed_base=0)
    for c, t0 in enumerate(range(0, steps, K)):
        eng.step(K, actions=None, philox_seed=31, env_base=0, step_base=t0, reward=rew, done=done, obs=obs,
                 ev_act=ev[0], ev_watch=ev[1], ev_misc=evm, auto_reset=True)
        sl = slice(c * K, (c + 1) * K)
        assert np.array_equal(rew.cpu().numpy(), got['reward'][sl]), f'{cfg} rewards, steps {t0}..{t0 + K}'
        assert np.array_equal(done.cpu().numpy(), got['done'][sl]), f'{cfg} done, steps {t0}..{t0 + K}'
    assert np.array_equal(obs.cpu().numpy().view(np.uint64), got['obs'].view(np.uint64)), f'{cfg} obs, last call'
    assert np.array_equal(eng.export_state().cpu().numpy(), got['state']), f'{cfg} state records'
    assert float(got['episodes'][0]) == float(got['done'].sum())  # the metrics all-reduce summed both ranks
    eng.close()


@pytest.mark.timeout(600)
def test_bench_launcher_two_ranks_share_gpu(tmp_path):
    """bench.py --gpus 2 without an external launcher: a GPU-free parent starts two rank processes (gloo, both on
    GPU 0 under MFG_BENCH_SHARE_GPU=1) and re-prints rank 0's line, which must report 2 ranks."""
    if not gpu_available():
        pytest.skip('no GPU')
    env = dict(os.environ, MFG_BENCH_SHARE_GPU='1')
    r = subprocess.run([sys.executable, str(ROOT / 'bench.py'), '--gpus', '2', '--backend', 'gloo', '--batch', '4096',
                        '--warmup', '16', '--steps', '32', '--alt-steps', '0', '--packed-steps', '0',
                        '--no-cpu-baseline', '--rank-timeout', '400'], env=env, capture_output=True, text=True,
                       timeout=500)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith('{')][-1])
    assert line['n_gpus'] == 2 and line['backend'] == 'gloo' and line['n_ranks_gloo'] == 2 and 'launcher' in line
    assert 'n_ranks_rccl' not in line  # a gloo group is not labelled RCCL
    assert line['config']['global_batch'] == 2 * 4096 and line['value'] > 0


def test_bench_default_lines_run(tmp_path):
    """bench.py with its default lines (f64 headline, the other obs dtype, packed entries, fused projection,
    dense f32 + projection GEMM, CPU baseline) on a small batch: the run the driver makes, shortened. Every side
    line must be present and positive (a dtype mismatch in one of them once crashed the default run)."""
    if not gpu_available():
        pytest.skip('no GPU')
    r = subprocess.run([sys.executable, str(ROOT / 'bench.py'), '--batch', '4096', '--warmup', '16', '--steps', '32',
                        '--cpu-seconds', '1'], capture_output=True, text=True, timeout=500)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith('{')][-1])
    assert line['value'] > 0 and 'f64 obs' in line['dtype']
    assert line['alt_obs_dtype']['value'] > 0 and line['alt_obs_dtype']['obs'] == 'f32'
    p = line['packed_obs']
    assert p['value'] > 0 and p['fused_proj']['value'] > 0 and p['dense_f32_plus_proj']['value'] > 0
    assert line['cpu_baseline']['value'] > 0 and line['cpu_baseline']['cores'] >= 1
    assert line['roofline']['frac'] > 0 and 'frac_sec8d' not in line['roofline'] and line['parity']['timed_mode_test']
    assert line['roofline']['peak_measured'] > 1000  # the HIP copy kernel's GB/s
    assert line['backend'] is None and line['n_ranks_rccl'] is None  # bare single process: no group


@pytest.mark.timeout(600)
def test_bench_under_torchrun_one_rank_joins_rccl(tmp_path):
    """The driver's launch form at N = 1: `python -m torch.distributed.run --nproc-per-node 1 bench.py --gpus 1`,
    started as a fresh child process (nothing on the GPU in this process's child before the launcher). The rank must
    join a real nccl (RCCL) process group and run the barriers and the MAX / metrics all-reduces on device tensors."""
    if not gpu_available():
        pytest.skip('no GPU')
    env = dict(os.environ)
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
    out = tmp_path / 'line.json'
    r = subprocess.run([sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '1',
                        '--master-addr', '127.0.0.1', '--master-port', str(_free_port()), str(ROOT / 'bench.py'),
                        '--gpus', '1', '--batch', '4096', '--warmup', '16', '--steps', '32', '--alt-steps', '0',
                        '--packed-steps', '0', '--no-cpu-baseline'], env=env, capture_output=True, text=True,
                       timeout=500)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith('{')][-1])
    out.write_text(json.dumps(line))
    assert line['backend'] == 'nccl' and line['n_ranks_rccl'] == 1 and line['n_gpus'] == 1
    c = line['collectives']
    assert c['tensors'].startswith('cuda') and c['metrics_allreduce_episodes'] >= 0
    assert line['value'] > 0

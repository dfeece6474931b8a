#!/usr/bin/env python3
"""bench.py — env-steps/sec of the MI355X batched step engine on the headline workload.

Workload (BASELINE.json configs[2]): 'large' level, 8 agents, doors + items + batteries,
B = 65536 envs per GPU, synthetic uniform random actions (Philox4x32-10 on the device), auto-reset with
reference reset semantics, dense fp32 observations (8 agents x 7 layers x 7x7) written to HBM every step,
f64 rewards, done flags and info events. One "step" = one env-step of every env on every GPU.

Timed region: exactly --steps steps (fused into launches of --fuse steps), bracketed by barrier +
torch.cuda.synchronize() on both sides, max over ranks. value = all envs x steps / max time.
roofline: the step kernel's algorithmic bytes (11,391 B per env-step, fp32 obs) per
launch / its mean launch time measured with HIP events on the launch stream; peak 8 TB/s (HBM3E).
cpu_baseline: the C restatement (oracle/, kind "port") on this host's cores, same config and actions,
bounded sample. Multi-GPU: `python -m torch.distributed.run --nproc-per-node N bench.py --gpus N`,
one rank per GPU, env ranges sharded (weak scaling), no collective in the data path.
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
for _p in (ROOT / 'marl-factory-grid_amd', ROOT / 'oracle', ROOT / 'tests'):
    if str(_p) not in sys.path:
        sys.path.insert(0, str(_p))

ALGO_BYTES_PER_ENV_STEP = 11391  # 415 B state/IO + 10,976 B dense fp32 obs (C3)
HBM_PEAK_GBS = 8000.0            # MI355X HBM3E spec (MI355X_MICROARCH.md)
METRIC = "env-steps/sec (whole node), 8-agent 'large' level, batch 65536, 1/2/4/8 MI355X"


def cpu_baseline(config, seconds, workers, seed):
    """Time the C port (oracle) on host cores: `workers` processes, each stepping its own envs."""
    import multiprocessing as mp
    ctx = mp.get_context('fork')
    q = ctx.Queue()
    procs = [ctx.Process(target=_cpu_worker, args=(config, seconds, seed, w, q)) for w in range(workers)]
    for p in procs:
        p.start()
    res = [q.get() for _ in procs]
    for p in procs:
        p.join()
    steps = sum(r[0] for r in res)
    wall = max(r[1] for r in res)
    return steps / wall, steps, wall


def _cpu_worker(config, seconds, seed, w, q):
    import numpy as np
    import oracle as O
    from philox import synthetic_actions
    from mfg_amd.spec import compile_spec
    spec = compile_spec(config)
    env = O.OracleEnv(spec, 10_000_000 + w)
    env.reset()
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for _ in range(25):
            a = synthetic_actions(seed, [w], n, spec.n_actions)[0]
            _, d, _ = env.step(a)
            n += 1
            if d:
                env.reset()
    q.put((n, time.perf_counter() - t0))


def load_pmc(config_tag):
    """HBM traffic per step-kernel launch from the committed rocprofv3 PMC summary (profiles/)."""
    for p in sorted((ROOT / 'profiles').glob('pmc_*.json'), reverse=True):
        try:
            d = json.loads(p.read_text())
        except Exception:
            continue
        if d.get('workload') == config_tag:
            return d
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=200)
    ap.add_argument('--warmup', type=int, default=40)
    ap.add_argument('--fuse', type=int, default=8, help='env-steps fused per kernel launch')
    ap.add_argument('--batch', type=int, default=65536, help='envs per GPU')
    ap.add_argument('--config', default='large8.yaml')
    ap.add_argument('--cpu-seconds', type=float, default=12.0)
    ap.add_argument('--cpu-workers', type=int, default=0, help='0 = min(16, host cores)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1:
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        torch.cuda.set_device(local)
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    from mfg_amd.spec import compile_spec
    from mfg_amd.engine import Engine

    spec = compile_spec(args.config)
    B, A, F = args.batch, spec.n_agents, args.fuse
    dev = torch.device('cuda', local)
    eng = Engine(spec, B, device=local)
    env_base = rank * B
    obs = torch.zeros((F,) + eng.obs_shape(), dtype=torch.float32, device=dev)
    rew = torch.zeros((F, B, A), dtype=torch.float64, device=dev)
    done = torch.zeros((F, B), dtype=torch.uint8, device=dev)
    ev_a = torch.zeros((F, B, A), dtype=torch.uint8, device=dev)
    ev_w = torch.zeros((F, B, A), dtype=torch.uint8, device=dev)
    ev_m = torch.zeros((F, B, 10), dtype=torch.int32, device=dev)
    eng.reset(obs=obs[0], init=True, seed_base=env_base)
    stream = torch.cuda.current_stream(dev)
    step_no = 0

    def run(n, events=None):
        nonlocal step_no
        done_steps = 0
        while done_steps < n:
            k = min(F, n - done_steps)
            if events is not None:
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record(stream)
            eng.step(k, actions=None, philox_seed=12345, env_base=env_base, step_base=step_no, reward=rew, done=done,
                     obs=obs, ev_act=ev_a, ev_watch=ev_w, ev_misc=ev_m, auto_reset=True)
            if events is not None:
                e.record(stream)
                events.append((s, e, k))
            step_no += k
            done_steps += k

    run(args.warmup)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    launches = []
    t0 = time.perf_counter()
    run(args.steps, launches)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    full = [(s.elapsed_time(e) * 1e-3, k) for s, e, k in launches if k == F] or \
           [(s.elapsed_time(e) * 1e-3, k) for s, e, k in launches]
    mean_launch = sum(t for t, _ in full) / len(full)
    k_launch = full[0][1]
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        m = torch.tensor([float(done[:].sum().item())], dtype=torch.float64, device=dev)
        dist.all_reduce(m)  # optional metrics all-reduce (tiny, latency-bound)
    total = B * world * args.steps
    value = total / elapsed
    if rank == 0:
        algo = ALGO_BYTES_PER_ENV_STEP * B * k_launch
        achieved = algo / mean_launch / 1e9
        pmc = load_pmc('large8_b65536') if args.config == 'large8.yaml' and B == 65536 else None
        traffic = None
        if pmc and pmc.get('fuse') == k_launch:
            traffic = pmc.get('hbm_bytes_per_launch')
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            workers = args.cpu_workers or min(16, len(os.sched_getaffinity(0)))
            v, n, wall = cpu_baseline(args.config, args.cpu_seconds, workers, 12345)
            cpu = {"value": round(v, 1), "unit": "env-steps/s", "cores": workers, "kind": "port",
                   "sample": f"{n} env-steps of {args.config} (obs incl.) on {workers} processes x "
                             f"{wall:.1f}s, C restatement oracle/mfg_oracle.c"}
        out = {
            "metric": METRIC, "value": round(value, 1), "unit": "env-steps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (Philox4x32-10 uniform random actions, device-side)",
            "config": {"workload": "C3 large8: 'large' level, 8 agents, doors+items+batteries, pomdp_r 3",
                       "envs_per_gpu": B, "global_batch": B * world, "obs": "dense fp32 [8,7,7,7] per env-step",
                       "fuse": F, "auto_reset": True, "parallelism": f"env-shard x{world}"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                         "kernel": "k_step", "algo_bytes_per_env_step": ALGO_BYTES_PER_ENV_STEP,
                         "mean_launch_ms": round(mean_launch * 1e3, 3), "env_steps_per_launch": B * k_launch},
            "cpu_baseline": cpu,
        }
        print(json.dumps(out))
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()

#!/usr/bin/env python3
"""bench.py — env-steps/sec of the MI355X batched step engine on the headline workload.

Workload (BASELINE.json configs[2]): 'large' level, 8 agents, doors + items + batteries,
B = 65536 envs per GPU, synthetic uniform random actions (Philox4x32-10 on the device, keyed (seed, env)
at counter (step, agent)), auto-reset with reference reset semantics, dense fp32 observations
(8 agents x 7 layers x 7x7) written to HBM every step, f64 rewards, done flags and info events.
One "step" = one env-step of every env on every GPU. Measurement protocol of SURVEY §8(d): >= 600
warm-up steps (every env has passed episode 1, Q11/Q12 active), then >= 2000 timed steps; with
500-step episodes the timed window holds the resets in proportion.

Timed region: exactly --steps steps (mfg_step calls of --fuse steps), bracketed by barrier +
torch.cuda.synchronize() on both sides, max over ranks. value = all envs x steps / max time.

roofline: per-kernel HIP events recorded by the engine around each launch on the launch stream
(mfg_profile) over the timed region. Top level = the dominant kernel (largest share of time) with its
algorithmic bytes per launch; "pipeline" = the whole step against SURVEY §8(d)'s
11,391 B per env-step; "kernels" = every kernel's share. traffic = HBM bytes per launch of the dominant
kernel from the committed rocprofv3 PMC summary (profiles/pmc_*.json, FETCH_SIZE x2 + WRITE_SIZE).
cpu_baseline: the C restatement (oracle/, kind "port") on this host's cores, same config and actions,
bounded sample.

Multi-GPU (weak scaling, env ranges sharded, no collective in the data path): either the driver's
`python -m torch.distributed.run --nproc-per-node N bench.py --gpus N`, or plain `python bench.py --gpus N`,
which starts the N rank processes itself (launch_ranks) before anything touches the GPU and prints rank 0's
line. Under a launcher (WORLD_SIZE set, N = 1 included) every rank joins one process group (nccl = RCCL) whose size
must equal --gpus; the line reports `backend` and `n_ranks_rccl` (nccl groups only; gloo lines say `n_ranks_gloo`),
and the barrier, the MAX all-reduce of the elapsed time and the metrics all-reduce run on that group.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
for _p in (ROOT / 'marl-factory-grid_amd', ROOT / 'oracle', ROOT / 'tests'):
    if str(_p) not in sys.path:
        sys.path.insert(0, str(_p))

ALGO_BYTES_PER_ENV_STEP = 11391  # 415 B state/IO + 10,976 B dense fp32 obs (C3); f64 obs: 22,367
PARITY_TESTS = {  # the GPU tests that pin the exact mode each line times (tests/test_gpu_timed_path.py)
    'f64': 'tests/test_gpu_timed_path.py::test_timed_path_k8_f64_b65536_matches_oracle',
    'f32': 'tests/test_gpu_timed_path.py::test_timed_path_k8_fp32_b65536_matches_oracle'}
HBM_PEAK_GBS = 8000.0            # MI355X HBM3E spec (MI355X_MICROARCH.md)
CU_CLOCK_HZ, N_CU = 2.4e9, 256   # MI355X: 256 CUs, 2.4 GHz peak engine clock (MI355X_MICROARCH.md)
METRIC = "env-steps/sec (whole node), 8-agent 'large' level, batch 65536, 1/2/4/8 MI355X"


def core_bytes(spec):
    """SURVEY §8(d) canonical minimal SoA bytes per env-step without the obs: mutable state read + written
    (agent pos u16, door open+timer u8, item/dirt positions u16, battery and dirt amounts f64, 7 B of
    counters), per-episode constants read (pod/drop-off/destination/machine/maintainer positions, frozen
    ray origins u16, frozen battery f64, entity ids i32), actions u8, reward f64, done u8. C3: 415 B."""
    from mfg_amd import abi
    c = spec.c
    A = spec.n_agents
    q = {int(r.op): r for r in c.rules[:c.n_rules]}

    def spawn(op):
        return int(q[op].i[0]) if op in q else 0
    bat = 8 * A if abi.RULE_SPAWN_BATTERIES in q else 0
    mut = 2 * A + c.n_doors + 2 * spawn(abi.RULE_SPAWN_ITEMS) + bat + 7
    if c.has_dirt:
        mut += 10 * int(c.dirt_quantity)
    const = 2 * A + bat + 4 * A
    for op in (abi.RULE_SPAWN_PODS, abi.RULE_SPAWN_DROPOFFS, abi.RULE_SPAWN_DESTS, abi.RULE_SPAWN_MACHINES,
               abi.RULE_SPAWN_MAINTAINERS):
        const += 2 * spawn(op)
    return 2 * mut + const + A + 8 * A + 1


def issue_floors(c, launch_ms):
    """Issue-unit floors of one launch from its PMC instruction counts (chip totals per dispatch), at 2.4 GHz
    on 256 CUs: VALU = INSTS_VALU x 2 cycles (a wave64 op on a SIMD-32) over 4 SIMDs per CU; SALU =
    INSTS_SALU x 1 cycle on the CU's one scalar unit; LDS = SQ_LDS_IDX_ACTIVE (LDS-array cycles, bank-conflict
    extras included). The binding unit is the largest floor; frac = floor / measured launch time."""
    cyc = CU_CLOCK_HZ * N_CU
    floors = {"valu": c['SQ_INSTS_VALU'] * 2 / (4 * cyc) * 1e3, "salu": c['SQ_INSTS_SALU'] / cyc * 1e3}
    if c.get('SQ_LDS_IDX_ACTIVE') is not None:
        floors["lds"] = c['SQ_LDS_IDX_ACTIVE'] / cyc * 1e3
    unit = max(floors, key=floors.get)
    return {"unit": unit, "frac": round(floors[unit] / launch_ms, 3),
            "floors_ms": {k: round(v, 4) for k, v in floors.items()},
            "frac_by_unit": {k: round(v / launch_ms, 3) for k, v in floors.items()}}


def algo_bytes(kernel, spec, obs_bytes_per_env, k_launch):
    """Algorithmic (minimal) bytes one launch of `kernel` moves per env."""
    core = core_bytes(spec)
    if kernel == 'k_logic':
        return core
    if kernel == 'k_obs':
        return obs_bytes_per_env + 230  # obs written once + mutable/constant state read once
    if kernel == 'k_replay':
        return 2 * (4 * 624 + 2 * spec.c.n_floor)  # MT state + floor permutation, read + written
    return None


def cgroup_cpus():
    """CPUs the cgroup v2 quota allows (cpu.max 'quota period'), or None without a quota."""
    try:
        q, per = open('/sys/fs/cgroup/cpu.max').read().split()[:2]
        return None if q == 'max' else max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        return None


def cpu_baseline(config, seconds, workers, seed):
    """Time the C port (oracle) on host cores: `workers` processes, each stepping its own env."""
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
    import numpy as np  # noqa: F401
    import oracle as O
    from philox import synthetic_actions
    from mfg_amd.spec import compile_spec
    spec = compile_spec(config)
    env = O.OracleEnv(spec, w)
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


def cpu_model():
    try:
        for line in open('/proc/cpuinfo'):
            if line.startswith('model name'):
                return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return 'unknown'


def stream_copy_gbs(dev, nbytes=2 << 30, reps=10):
    """Measured HBM stream-copy bandwidth on this GPU: the library's hand-written 16-B-per-lane copy
    kernel (mfg_hbm_copy) over `nbytes` moves 2 x nbytes; best of `reps` after a warm-up, timed with events on the
    stream the kernel is launched on. torch's copy_ is reported beside it (it measured ~4.5 TB/s in round 4)."""
    import torch
    from mfg_amd.engine import hbm_copy
    a = torch.empty(nbytes // 4, dtype=torch.float32, device=dev)
    b = torch.empty_like(a)
    a.fill_(1.0)
    stream = torch.cuda.current_stream(dev)
    res = {}
    for name, fn in (('hip_copy16', lambda: hbm_copy(b, a, stream)), ('torch_copy_', lambda: b.copy_(a))):
        fn()
        best = None
        for _ in range(reps):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record(stream)
            fn()
            e.record(stream)
            e.synchronize()
            t = s.elapsed_time(e) * 1e-3
            best = t if best is None else min(best, t)
        res[name] = round(2 * nbytes / best / 1e9, 1)
    del a, b
    torch.cuda.empty_cache()
    return res


def load_pmc(workload):
    """HBM traffic per launch from the committed rocprofv3 PMC summary (profiles/pmc_*.json)."""
    for p in sorted((ROOT / 'profiles').glob('pmc_*.json'), reverse=True):
        try:
            d = json.loads(p.read_text())
        except Exception:
            continue
        if d.get('workload') == workload:
            return d
    return None


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n, argv, share_gpu=False, dry_run=False, rank_timeout=900.0):
    """`bench.py --gpus N` (N > 1) started without a torch.distributed launcher: run N rank processes of this
    script, one per GPU, and print rank 0's JSON line. The parent stays GPU-free: it only counts devices
    (torch.cuda.device_count() does not initialise HIP on this image) and starts each rank as a child process
    with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set, as torch.distributed.run would.
    If any rank fails the others are killed (by their own Popen handles) and the largest exit code returned; if
    the ranks are still running after `rank_timeout` seconds (an RCCL init or barrier hang), all are killed and
    124 is returned."""
    if not (share_gpu or dry_run):
        import torch
        visible = torch.cuda.device_count()
        if visible < n:
            print(f"bench.py: {n} GPUs requested, {visible} visible", file=sys.stderr)
            return 2
    port = _free_port()
    out = tempfile.NamedTemporaryFile(prefix='bench_rank0_', suffix='.out', delete=False)
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK='0', MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
        env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')  # dmabuf IPC only on this pool (RCCL)
        procs.append(subprocess.Popen([sys.executable, '-u', str(Path(__file__).resolve())] + list(argv), env=env,
                                      stdout=out if r == 0 else subprocess.DEVNULL))
    rc = 0
    t_start = time.monotonic()
    while procs:
        time.sleep(0.2)
        if time.monotonic() - t_start > rank_timeout:
            print(f"bench.py: ranks still running after {rank_timeout:.0f}s, killing them", file=sys.stderr)
            for q in procs:
                q.kill()
            for q in procs:
                q.wait()
            procs = []
            rc = 124
            break
        for p in list(procs):
            code = p.poll()
            if code is None:
                continue
            procs.remove(p)
            if code != 0:
                rc = max(rc, code if code > 0 else 128 - code)
                for q in procs:
                    q.kill()
                for q in procs:
                    q.wait()
                procs = []
                break
    out.close()
    lines = [ln for ln in Path(out.name).read_text().splitlines() if ln.startswith('{')]
    os.unlink(out.name)
    if rc == 0 and lines:
        d = json.loads(lines[-1])
        d["launcher"] = f"bench.py --gpus {n}: {n} rank processes spawned by a GPU-free parent"
        print(json.dumps(d), flush=True)
    elif rc == 0:
        print("bench.py: rank 0 printed no result line", file=sys.stderr)
        rc = 1
    return rc


def init_ranks(args):
    """(world, rank, local, n_ranks, backend) of this process. Under a launcher (WORLD_SIZE set, e.g. the driver's
    `torch.distributed.run --nproc-per-node N`, N = 1 included) every rank joins one process group (nccl = RCCL unless
    --backend says otherwise) and checks that its world size equals --gpus; a bare single-process run has no group
    (backend None)."""
    launched = 'WORLD_SIZE' in os.environ
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if (args.gpus > 1 or launched) and world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if not launched:
        return world, rank, local, 1, None
    import torch
    import torch.distributed as dist
    os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
    if args.dry_run:
        dist.init_process_group('gloo')
    else:
        if os.environ.get('MFG_BENCH_SHARE_GPU') == '1':  # rehearsal of N ranks on fewer GPUs (not a bench number)
            local = local % torch.cuda.device_count()
        torch.cuda.set_device(local)
        if args.backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
        else:
            dist.init_process_group(args.backend)
    n_ranks = dist.get_world_size()
    if n_ranks != world or n_ranks != args.gpus:
        raise SystemExit(f"bench.py: process group has {n_ranks} ranks, expected {world} (--gpus {args.gpus})")
    return world, rank, local, n_ranks, dist.get_backend()


def rank_fields(n_ranks, backend):
    """How the line's ranks were joined: n_ranks_rccl only for an nccl (= RCCL on ROCm) group."""
    f = {"backend": backend}
    if backend == 'nccl':
        f["n_ranks_rccl"] = n_ranks
    elif backend is not None:
        f[f"n_ranks_{backend}"] = n_ranks
    else:
        f["n_ranks_rccl"] = None
        f["process_group"] = "none (single process, not started by a launcher)"
    return f


def dry_run(args, world, rank, n_ranks, backend):
    """CPU rehearsal of the multi-rank protocol (no GPU, gloo): env ranges, barrier-bracketed timed region,
    MAX over ranks and the metrics all-reduce, with the same output fields as the GPU line."""
    import torch
    import torch.distributed as dist
    from mfg_amd.shard import env_range, allreduce_metrics
    B = args.batch
    first, count = env_range(rank, world, B)
    if backend:
        dist.barrier()
    t0 = time.perf_counter()
    acc = 0
    for _ in range(args.steps):
        acc += count
    elapsed = time.perf_counter() - t0 + 1e-3 * (rank + 1)
    if backend:
        dist.barrier()
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    m = allreduce_metrics(torch.tensor([float(acc)], dtype=torch.float64))
    ranges = [None] * world
    if backend:
        dist.all_gather_object(ranges, (first, count))
    else:
        ranges = [(first, count)]
    if rank == 0:
        print(json.dumps({"metric": METRIC, "dry_run": True, "value": B * world * args.steps / elapsed,
                          "n_gpus": world, **rank_fields(n_ranks, backend), "steps": args.steps, "max_elapsed_s": elapsed,
                          "env_ranges": ranges, "metrics_allreduce": float(m[0])}), flush=True)
    if backend:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=2000)
    ap.add_argument('--warmup', type=int, default=600)
    ap.add_argument('--fuse', type=int, default=8, help='env-steps per mfg_step call (one k_replay per call)')
    ap.add_argument('--batch', type=int, default=65536, help='envs per GPU')
    ap.add_argument('--config', default='large8.yaml')
    ap.add_argument('--cpu-seconds', type=float, default=12.0)
    ap.add_argument('--cpu-workers', type=int, default=0,
                    help='0 = the usable cores: min(affinity, cgroup cpu.max quota)')
    ap.add_argument('--obs-dtype', choices=['f32', 'f64'], default='f64',
                    help='obs precision of the headline line: f64, the reference\'s own (Q25, '
                         'utils/observation_builder.py:162); f32 is the alt_obs_dtype side line')
    ap.add_argument('--alt-steps', type=int, default=None,
                    help='steps of the second measurement with the other obs dtype (default: --steps; 0 = off)')
    ap.add_argument('--packed-steps', type=int, default=None,
                    help='steps of each packed-obs measurement (entries; entries + fused projection; dense + GEMM) (default: --steps; 0 = off)')
    ap.add_argument('--cap', type=int, default=32, help='packed entries stored per agent row')
    ap.add_argument('--emb', type=int, default=96, help='fused projection width (obs_emb_size of RecurrentAC)')
    ap.add_argument('--backend', default='nccl', help="torch.distributed backend for N > 1 ('nccl' = RCCL)")
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--rank-timeout', type=float, default=900.0,
                    help='bench.py --gpus N as its own launcher: kill the ranks after this many seconds')
    ap.add_argument('--no-profile', action='store_true', help='no per-kernel HIP events in the timed region')
    ap.add_argument('--serial', action='store_true',
                    help='attribution run: every kernel on one stream (mfg_variant.serial), so per-kernel times '
                         'exclude the second stream\'s overlap (C4); not a headline line')
    ap.add_argument('--dry-run', action='store_true',
                    help='CPU rehearsal of the rank protocol (gloo, no GPU, no engine); not a bench number')
    args = ap.parse_args()

    if args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        return launch_ranks(args.gpus, sys.argv[1:], share_gpu=os.environ.get('MFG_BENCH_SHARE_GPU') == '1',
                            dry_run=args.dry_run, rank_timeout=args.rank_timeout)
    world, rank, local, n_ranks, backend = init_ranks(args)
    if args.dry_run:
        return dry_run(args, world, rank, n_ranks, backend)

    import torch
    import torch.distributed as dist
    from mfg_amd.spec import compile_spec
    from mfg_amd.engine import Engine, EV_MISC
    from mfg_amd.shard import env_range

    spec = compile_spec(args.config)
    B, A, F = args.batch, spec.n_agents, args.fuse
    dev = torch.device('cuda', local)
    eng = Engine(spec, B, device=local, variant={'serial': 1} if args.serial else None)
    env_base, _ = env_range(rank, world, B)
    obs_t = torch.float64 if args.obs_dtype == 'f64' else torch.float32
    obs = torch.zeros((F,) + eng.obs_shape(), dtype=obs_t, device=dev)
    rew = torch.zeros((F, B, A), dtype=torch.float64, device=dev)
    done = torch.zeros((F, B), dtype=torch.uint8, device=dev)
    ev_a = torch.zeros((F, B, A), dtype=torch.uint8, device=dev)
    ev_w = torch.zeros((F, B, A), dtype=torch.uint8, device=dev)
    ev_m = torch.zeros((F, B, EV_MISC), dtype=torch.int32, device=dev)
    eng.reset(obs=obs[0], init=True, seed_base=env_base)
    stream = torch.cuda.current_stream(dev)
    step_no = 0
    red_dev = dev if backend in (None, 'nccl') else torch.device('cpu')  # gloo reduces host tensors
    episodes = torch.zeros((), dtype=torch.float64, device=red_dev)

    def run(n, events=None, profile=False, obs_buf=None, after=None):
        """n steps in calls of F (the last call may be shorter). Per-kernel HIP events are recorded only
        around full-K calls, so the per-launch roofline figures are always those of K=F launches.
        after(k): work run on the stream after each call (the dense obs consumer of the packed comparison)."""
        nonlocal step_no
        done_steps = 0
        while done_steps < n:
            k = min(F, n - done_steps)
            if profile:
                eng.profile(k == F)
            if events is not None:
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record(stream)
            eng.step(k, actions=None, philox_seed=12345, env_base=env_base, step_base=step_no, reward=rew, done=done,
                     obs=obs if obs_buf is None else obs_buf, ev_act=ev_a, ev_watch=ev_w, ev_misc=ev_m,
                     auto_reset=True)
            if after is not None:
                after(k)
            if events is not None:
                e.record(stream)
                events.append((s, e, k))
            step_no += k
            done_steps += k

    run(args.warmup)
    torch.cuda.synchronize(dev)
    if backend:
        dist.barrier()
    torch.cuda.synchronize(dev)
    calls = []
    eng.profile_read()
    t0 = time.perf_counter()
    run(args.steps, calls, profile=not args.no_profile)
    torch.cuda.synchronize(dev)
    if backend:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    prof = eng.profile_read()
    eng.profile(False)
    if backend:
        t = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        episodes += done.double().sum().to(red_dev)
        dist.all_reduce(episodes)  # optional metrics all-reduce (tiny, latency-bound)
    total = B * world * args.steps
    value = total / elapsed
    def timed(n, obs_buf, after=None):
        """n more steps into obs_buf, timed like the headline (barrier + synchronize brackets, max over ranks)."""
        run(F, obs_buf=obs_buf, after=after)
        torch.cuda.synchronize(dev)
        if backend:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        run(n, obs_buf=obs_buf, after=after)
        torch.cuda.synchronize(dev)
        if backend:
            dist.barrier()
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t1
        if backend:
            t = torch.tensor([el], dtype=torch.float64, device=red_dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el

    # the same workload with the other obs precision (the reference's own obs are f64, Q25), timed the same way
    alt = None
    alt_steps = args.steps if args.alt_steps is None else args.alt_steps
    if alt_steps > 0:
        alt_dtype = 'f32' if args.obs_dtype == 'f64' else 'f64'
        obs_alt = torch.zeros((F,) + eng.obs_shape(), dtype=torch.float64 if alt_dtype == 'f64' else torch.float32,
                              device=dev)
        el2 = timed(alt_steps, obs_alt)
        alt_obs_bytes = sum(spec.n_layers) * spec.obs_hw[0] * spec.obs_hw[1] * (8 if alt_dtype == 'f64' else 4)
        alt_step_bytes = core_bytes(spec) + alt_obs_bytes
        alt_value = B * world * alt_steps / el2
        alt = {"obs": alt_dtype, "value": round(alt_value, 1), "unit": "env-steps/s", "steps": alt_steps,
               "ms_per_step": round(el2 / alt_steps * 1e3, 4), "algo_bytes_per_env_step": alt_step_bytes,
               "pipeline_GBs": round(alt_value / world * alt_step_bytes / 1e9, 2),
               "pipeline_frac": round(alt_value / world * alt_step_bytes / 1e9 / HBM_PEAK_GBS, 5)}
        del obs_alt
    # packed obs: the nonzero entries per agent row instead of the dense obs; beside it the same
    # with the policy-input projection fused into the render, and what that replaces (dense obs + one GEMM)
    packed = None
    packed_steps = args.steps if args.packed_steps is None else args.packed_steps
    if packed_steps > 0:
        from mfg_amd.engine import PackedObs
        kdim = eng.lmax * eng.obs_hw[0] * eng.obs_hw[1]
        dense_bytes = core_bytes(spec) + sum(spec.n_layers) * spec.obs_hw[0] * spec.obs_hw[1] * 4
        pe = PackedObs(eng, K=F, cap=args.cap)
        el5 = timed(packed_steps, pe)
        ev = B * world * packed_steps / el5
        pe_bytes = core_bytes(spec) + A * (4 + 6 * args.cap)
        max_nnz = int(pe.count.max())
        del pe
        g = torch.Generator(device=dev).manual_seed(0)
        w = torch.randn((args.emb, kdim), generator=g, device=dev) * 0.05
        po = PackedObs(eng, K=F, cap=args.cap, weight=w, bias=torch.zeros(args.emb, device=dev))
        el3 = timed(packed_steps, po)
        pk_bytes = pe_bytes + A * 4 * args.emb
        pv = B * world * packed_steps / el3
        del po
        # what the fused projection replaces: dense f32 obs + the policy's obs_proj over them (one GEMM per call on
        # the same stream, hipBLASLt), i.e. the policy input from materialised obs
        emb_d = torch.empty((F * B * A, args.emb), device=dev)
        wt = w.t().contiguous()
        # dense f32 obs (the policy's input precision) whatever the headline's obs dtype
        obs32 = obs if obs.dtype == torch.float32 else torch.zeros((F,) + eng.obs_shape(), dtype=torch.float32,
                                                                   device=dev)

        def proj(k):
            torch.matmul(obs32[:k].reshape(k * B * A, -1), wt, out=emb_d[:k * B * A])
        el4 = timed(packed_steps, obs32, after=proj)
        dv = B * world * packed_steps / el4
        del emb_d, obs32
        packed = {"obs": f"packed entries (cap {args.cap}: u16 index + f32 value per nonzero, i32 count)",
                  "value": round(ev, 1), "unit": "env-steps/s", "steps": packed_steps,
                  "ms_per_step": round(el5 / packed_steps * 1e3, 4), "algo_bytes_per_env_step": pe_bytes,
                  "pipeline_GBs": round(ev / world * pe_bytes / 1e9, 2), "max_row_nnz": max_nnz,
                  "dense_f32_bytes_per_env_step": dense_bytes,
                  "fused_proj": {"obs": f"packed entries + fused obs_proj (E {args.emb}, f32)", "value": round(pv, 1),
                                 "ms_per_step": round(el3 / packed_steps * 1e3, 4), "algo_bytes_per_env_step": pk_bytes,
                                 "pipeline_GBs": round(pv / world * pk_bytes / 1e9, 2)},
                  "dense_f32_plus_proj": {"value": round(dv, 1), "ms_per_step": round(el4 / packed_steps * 1e3, 4),
                                          "what": "dense f32 obs, then obs_proj as one f32 GEMM per call"}}
    if rank == 0:
        full = [(s.elapsed_time(e) * 1e-3, k) for s, e, k in calls if k == F] or \
               [(s.elapsed_time(e) * 1e-3, k) for s, e, k in calls]
        mean_call = sum(t for t, _ in full) / len(full)
        k_call = full[0][1]
        obs_el = 8 if args.obs_dtype == 'f64' else 4
        obs_bytes = sum(spec.n_layers[a] for a in range(A)) * spec.obs_hw[0] * spec.obs_hw[1] * obs_el
        busy = sum(ms for ms, n in prof.values())
        kernels = {}
        for name, (ms, n) in prof.items():
            if not n:
                continue
            mean_ms = ms / n
            ab = algo_bytes(name, spec, obs_bytes, k_call)
            per_launch = None
            if ab is not None:
                units = B * (k_call if name == 'k_replay' else 1)
                per_launch = ab * (B if name == 'k_replay' else units)
            kernels[name] = {"launches": n, "mean_launch_ms": round(mean_ms, 4),
                             "share": round(ms / busy, 4) if busy else None,
                             "algo_bytes_per_launch": per_launch,
                             "achieved_GBs": round(per_launch / (mean_ms * 1e-3) / 1e9, 2) if per_launch else None}
        # resets beside the render (engine's second stream, reset_overlap): their launch time overlaps the main
        # stream's kernels, so what they cost the step is the step time the main stream's kernels leave unexplained
        aux = {'k_resetdone', 'k_obs_done'} if eng.layout.get('reset_overlap') else set()
        if aux & set(kernels):
            step_ms = elapsed / args.steps * 1e3
            main_ms = sum(ms for name, (ms, n) in prof.items() if name not in aux) / args.steps
            exposed = max(0.0, step_ms - main_ms)
            for name in aux & set(kernels):
                kernels[name]["stream"] = "aux"
                kernels[name]["ms_per_step"] = round(prof[name][0] / args.steps, 4)
            kernels["resets_exposed"] = {"ms_per_step": round(exposed, 4), "step_share": round(exposed / step_ms, 4),
                                         "how": "step time minus the main stream's kernel time per step (an upper "
                                                "bound: it includes launch gaps)"}
        dom = max((k for k in kernels if k in prof), key=lambda k: prof[k][0]) if kernels else None
        workload = f"{Path(args.config).stem}_b{B}_f{F}" + ('_f64' if args.obs_dtype == 'f64' else '')
        pmc = load_pmc(workload)
        traffic = None
        if pmc and dom and dom in pmc.get('hbm_bytes_per_launch', {}):
            traffic = pmc['hbm_bytes_per_launch'][dom]
        if pmc:  # issue rates per kernel from the committed PMC pass, against this run's launch time
            for name, kd in kernels.items():
                c = pmc.get('kernels', {}).get(name)
                if not c:
                    continue
                cu_cycles = kd["mean_launch_ms"] * 1e-3 * CU_CLOCK_HZ * N_CU
                kd["pmc"] = {"source": pmc.get('tag'),
                             "hbm_bytes_per_launch": round(c.get('hbm_bytes', 0)),
                             "traffic_over_algo": round(c['hbm_bytes'] / kd["algo_bytes_per_launch"], 3)
                             if kd.get("algo_bytes_per_launch") and c.get('hbm_bytes') else None,
                             "valu_per_cu_cycle": round(c['SQ_INSTS_VALU'] / cu_cycles, 3),
                             "salu_per_cu_cycle": round(c['SQ_INSTS_SALU'] / cu_cycles, 3),
                             "lds_per_cu_cycle": round(c['SQ_INSTS_LDS'] / cu_cycles, 3),
                             "wait_any_frac": c.get('wait_any_frac'),
                             "lds_array_busy": round(c['SQ_LDS_IDX_ACTIVE'] / cu_cycles, 3)
                             if c.get('SQ_LDS_IDX_ACTIVE') is not None else None,
                             "lds_bank_conflict_share": round(c['SQ_LDS_BANK_CONFLICT'] / c['SQ_LDS_IDX_ACTIVE'], 3)
                             if c.get('SQ_LDS_IDX_ACTIVE') else None}
                kd["issue"] = issue_floors(c, kd["mean_launch_ms"])
        step_bytes = core_bytes(spec) + obs_bytes  # C3: 415 + 10,976 = ALGO_BYTES_PER_ENV_STEP
        pipe_bytes = step_bytes * B * k_call
        if dom:
            dk = kernels[dom]
            achieved = dk["achieved_GBs"]
            roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBS, 5) if achieved else None, "traffic": traffic,
                    "kernel": dom, "mean_launch_ms": dk["mean_launch_ms"],
                    "algo_bytes_per_launch": dk["algo_bytes_per_launch"],
                    "pipeline": {"algo_bytes_per_env_step": step_bytes,
                                 "env_steps_per_call": B * k_call, "mean_call_ms": round(mean_call * 1e3, 3),
                                 "achieved": round(pipe_bytes / mean_call / 1e9, 2),
                                 "frac": round(pipe_bytes / mean_call / 1e9 / HBM_PEAK_GBS, 5)},
                    "kernels": kernels,
                    "issue": {k: v["issue"] for k, v in kernels.items() if "issue" in v},
                    "issue_how": "per kernel: VALU/SALU/LDS-array floors (ms) from the committed PMC pass "
                                 "(profiles/pmc_*.json) at 2.4 GHz x 256 CUs against this run's launch time; "
                                 "unit = the binding (largest) floor, frac = floor / launch time"}
        else:
            roof = {"bound": "hbm", "achieved": round(pipe_bytes / mean_call / 1e9, 2), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(pipe_bytes / mean_call / 1e9 / HBM_PEAK_GBS, 5),
                    "traffic": None, "kernel": "mfg_step pipeline", "mean_launch_ms": round(mean_call * 1e3, 3)}
        try:
            copies = stream_copy_gbs(dev)
        except RuntimeError:  # not enough free HBM for the 4 GiB copy pair
            copies = {}
        peak_meas = copies.get('hip_copy16')
        roof["peak_measured"] = peak_meas
        roof["peak_measured_how"] = ("hand-written 16-B-per-lane HIP copy kernel (mfg_hbm_copy) over 2 GiB, 2 x 2 GiB "
                                     f"moved, best of 10; torch copy_ of the same buffers: {copies.get('torch_copy_')} GB/s")
        if peak_meas and roof.get("achieved"):
            roof["frac_of_measured"] = round(roof["achieved"] / peak_meas, 5)
        if peak_meas and roof.get("pipeline"):
            roof["pipeline"]["frac_of_measured"] = round(roof["pipeline"]["achieved"] / peak_meas, 5)
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            visible = len(os.sched_getaffinity(0))
            quota = cgroup_cpus()
            usable = min(visible, quota) if quota else visible
            workers = args.cpu_workers or usable
            v, n, wall = cpu_baseline(args.config, args.cpu_seconds, workers, 12345)
            cpu = {"value": round(v, 1), "unit": "env-steps/s", "cores": workers, "kind": "port",
                   "per_core": round(v / workers, 1),
                   "cores_how": f"usable cores = min(affinity {visible}, cgroup cpu.max quota "
                                f"{quota if quota else 'none'}); worker sweep 1..128 on the GPU box saturates at the "
                                f"16-CPU quota (profiles/r04_cpu_sweep.json)",
                   "sample": f"{n} env-steps of {args.config} (obs incl., auto-reset) on {workers} processes x "
                             f"{wall:.1f}s, C restatement oracle/mfg_oracle.c, 1 env per process (independent "
                             f"envs: linear in cores up to the quota); {cpu_model()}"}
        out = {
            "metric": METRIC, "value": round(value, 1), "unit": "env-steps/s", "n_gpus": world,
            **rank_fields(n_ranks, backend),
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": f"f64 rewards/battery/dirt, {args.obs_dtype} obs",
            "data": "synthetic (Philox4x32-10 uniform random actions, device-side)",
            "config": {"workload": f"C3 {Path(args.config).stem}: 'large' level, 8 agents, doors+items+batteries, "
                                   f"pomdp_r 3" if args.config == 'large8.yaml' else Path(args.config).stem,
                       "envs_per_gpu": B, "global_batch": B * world,
                       "obs": f"dense {args.obs_dtype} per env-step ({obs_bytes} B)",
                       "fuse": F, "auto_reset": True, "parallelism": f"env-shard x{world}",
                       **({"serial": "attribution run: one stream, no reset/replay overlap"} if args.serial else {}),
                       "window": f"steps {args.warmup}..{args.warmup + args.steps} of every env" + (
                           "" if args.warmup + args.steps > 500 or args.config != 'large8.yaml' else
                           " (inside the first 500-step episode: no reset and no episode-2 obs path timed; the "
                           "default --warmup 600 --steps 2000 window times 4 episode ends)")},
            "roofline": roof,
            "parity": {"status": "bit-exact vs the C oracle, itself pinned by reference-generated fixtures",
                       "timed_mode_test": PARITY_TESTS[args.obs_dtype] if args.config == 'large8.yaml' else None,
                       "timed_mode": "K=8 mfg_step calls, Philox actions, auto-reset, B=65,536, 608 steps across the "
                                     "episode-500 reset; 256 envs vs their own oracle env every step (f64 rewards ==, "
                                     "done, events, obs bits), MT19937 + floor order after every call; every env of "
                                     "a quarter of the batch (all 65,536 in profiles/r05m_final_state_all_65536_envs"
                                     ".txt) vs the oracle's rollout: reward sums, episode ends, final MT + floor order",
                       "fixture_seeds": "tests/golden/large8_s{0,1}: reference step replayed through the C-ABI "
                                        "(tests/test_gpu_parity.py), py_seed 0 and 1",
                       "side_lines": {"alt_obs_dtype": PARITY_TESTS['f32' if args.obs_dtype == 'f64' else 'f64'],
                                      "packed_obs": "tests/test_marl.py (packed rows scatter to the dense f32 obs "
                                                    "bit-exactly)"}},
            "collectives": ({"tensors": str(red_dev), "barriers": "before and after every timed region",
                             "max_allreduce": "elapsed time of every timed region",
                             "metrics_allreduce_episodes": float(episodes.item())} if backend else None),
            "cpu_baseline": cpu,
            "alt_obs_dtype": alt,
            "packed_obs": packed,
        }
        print(json.dumps(out))
    eng.close()
    if backend:
        dist.destroy_process_group()


if __name__ == '__main__':
    sys.exit(main() or 0)

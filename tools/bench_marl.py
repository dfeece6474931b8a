#!/usr/bin/env python3
"""Throughput of the on-GPU A2C loop (mfg_amd.marl.BatchedA2C): env-steps/s of acting +
stepping + learning with packed obs and the fused projection, versus the same loop fed dense f32 obs (the
reference network's obs_proj on materialised obs). Prints one JSON line.
usage: python tools/bench_marl.py [--config large8.yaml] [--batch 8192] [--updates 20]
"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / 'marl-factory-grid_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='large8.yaml')
    ap.add_argument('--batch', type=int, default=8192)
    ap.add_argument('--updates', type=int, default=20)
    ap.add_argument('--n-steps', type=int, default=5)
    ap.add_argument('--eager', action='store_true', help='no HIP-graph capture of the update (BatchedA2C graph=False)')
    ap.add_argument('--act-graph', action='store_true', help='acting steps as HIP graphs (BatchedA2C act_graph=True)')
    ap.add_argument('--split-rows', type=int, default=0, help='marl.SPLIT_ROWS (rows per split-K GEMM batch)')
    args = ap.parse_args()
    import torch
    from mfg_amd.factory import BatchedFactory
    from mfg_amd.marl import BatchedA2C
    import mfg_amd.marl as M
    if args.split_rows:
        M.SPLIT_ROWS = args.split_rows
    f = BatchedFactory(args.config, args.batch, seed_base=0)
    tr = BatchedA2C(f, n_steps=args.n_steps, check_cap=True, graph=not args.eager, act_graph=args.act_graph)
    tr.train(3)  # warm-up (allocations, kernels; graph=True: two eager updates, then the capture)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    loss = tr.train(args.updates)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    steps = args.updates * args.n_steps
    tr.pobs.check()
    # the same engine work alone (K = 1 calls, packed obs + fused projection, random actions)
    acts = torch.zeros((args.batch, f.spec.n_agents), dtype=torch.int32, device=f.device)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for k in range(steps):
        f.engine.step(1, actions=acts, reward=tr.rew[0], done=tr.done[0], obs=tr.slot[1], auto_reset=True)
    torch.cuda.synchronize()
    env_el = time.perf_counter() - t1
    out = {"what": "on-GPU A2C (BatchedA2C): act + mfg_step(packed obs, fused obs_proj) + learn every n_steps",
           "update": "eager" if args.eager else "HIP graph (captured once, replayed per update)",
           "acting": "HIP graph per window slot" if args.act_graph else "eager",
           "split_rows": M.SPLIT_ROWS, "config": args.config, "envs": args.batch, "agents": f.spec.n_agents, "updates": args.updates,
           "n_steps": args.n_steps, "env_steps_per_s": round(args.batch * steps / el, 1),
           "agent_steps_per_s": round(args.batch * f.spec.n_agents * steps / el, 1),
           "ms_per_update": round(el / args.updates * 1e3, 3),
           "env_only_steps_per_s": round(args.batch * steps / env_el, 1), "final_loss": float(loss),
           "episodes": float(tr.episodes)}
    print(json.dumps(out))
    f.close()


if __name__ == '__main__':
    main()

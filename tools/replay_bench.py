#!/usr/bin/env python3
"""k_replay on a fixed workload (for ablations and exact variants): the same C3 state records (taken after a warm-up
of real steps) with the same shuffle debt in every env, replayed REPS times by mfg_replay; per-launch time from the
engine's HIP events (k_replay and its order kernels). Every variant starts from identical records, so timing-only
ablations that corrupt the permutation (NOSWAP, NOFWD, ...) cannot change the work the way they do inside a full
bench run (their broken permutations change the next episodes' dynamics and debts).
usage: MFG_HIP_LIB=<lib> python tools/replay_bench.py [--debt 69] [--reps 6]   (prints one JSON line)"""
import argparse
import hashlib
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / 'marl-factory-grid_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='large8.yaml')
    ap.add_argument('--batch', type=int, default=65536)
    ap.add_argument('--debt', type=int, default=69, help='floor shuffles per env (C3: 8.6 per env-step x K=8)')
    ap.add_argument('--warm-steps', type=int, default=48)
    ap.add_argument('--reps', type=int, default=6)
    args = ap.parse_args()
    import torch
    from mfg_amd.engine import HDR, Engine
    from mfg_amd.spec import compile_spec
    spec = compile_spec(args.config)
    eng = Engine(spec, args.batch, device=0)
    B, A = eng.B, eng.A
    dev = eng.device
    rew = torch.zeros((8, B, A), dtype=torch.float64, device=dev)
    done = torch.zeros((8, B), dtype=torch.uint8, device=dev)
    eng.reset(init=True, seed_base=0)
    for t0 in range(0, args.warm_steps, 8):
        eng.step(8, actions=None, philox_seed=12345, step_base=t0, reward=rew, done=done, auto_reset=True)
    st = eng.export_state()
    hdr = st.view(torch.int32)[:, eng.layout['o_hdr'] // 4:eng.layout['o_hdr'] // 4 + 40]
    hdr[:, HDR['debt']] = args.debt
    torch.cuda.synchronize()
    times, shas = [], set()
    stream = torch.cuda.current_stream(dev).cuda_stream
    for r in range(args.reps + 1):
        eng.import_state(st)
        torch.cuda.synchronize()
        eng.profile(True)
        eng.profile_read()
        t0 = time.perf_counter()
        rc = eng.L.mfg_replay(eng.h, stream)
        assert rc == 0, eng.L.mfg_last_error(eng.h)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        prof = eng.profile_read()
        eng.profile(False)
        if r:  # the first launch warms up
            times.append((prof['k_replay'][0], wall * 1e3))
        out = eng.export_state()
        shas.add(hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:16])
    ev = [t for t, _ in times]
    print(json.dumps({"lib": os.environ.get('MFG_HIP_LIB') or 'in-tree', "config": args.config, "envs": B,
                      "debt_shuffles_per_env": args.debt, "reps": args.reps,
                      "k_replay_ms_mean": round(sum(ev) / len(ev), 4), "k_replay_ms_min": round(min(ev), 4),
                      "k_replay_ms_max": round(max(ev), 4), "wall_ms_mean": round(sum(w for _, w in times) / len(times), 4),
                      "state_sha": sorted(shas), "deterministic": len(shas) == 1}))
    eng.close()


if __name__ == '__main__':
    main()

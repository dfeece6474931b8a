#!/usr/bin/env python3
"""Device time per phase of one on-GPU A2C update (BatchedA2C, C3, B envs): the T acting steps (policy forward +
sampling + mfg_step), the learner's forward (loss), backward, clip + RMSprop step, and the window slide, each
bracketed by HIP events on the stream (torch.cuda.Event). usage: python tools/prof_a2c_phases.py [--batch 8192]"""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / 'marl-factory-grid_amd'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='large8.yaml')
    ap.add_argument('--batch', type=int, default=8192)
    ap.add_argument('--updates', type=int, default=5)
    args = ap.parse_args()
    import torch
    import mfg_amd.marl as M
    from mfg_amd.factory import BatchedFactory
    f = BatchedFactory(args.config, args.batch, seed_base=0)
    tr = M.BatchedA2C(f, n_steps=5, check_cap=True)  # the bench's settings (cap 32)
    tr.train(2)
    torch.cuda.synchronize()
    acc = {}

    def ev():
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e
    for _ in range(args.updates):
        marks = [('start', ev())]
        learn, tr.learn = tr.learn, (lambda: None)
        for _ in range(tr.T):
            tr.step()
        tr.learn = learn
        marks.append(('act_5_steps', ev()))
        with torch.enable_grad():
            loss = tr.loss()
            marks.append(('loss_forward', ev()))
            tr.opt.zero_grad(set_to_none=True)
            loss.backward()
            marks.append(('backward', ev()))
            torch.nn.utils.clip_grad_norm_(tr.net.parameters(), 0.5)
            tr.opt.step()
            marks.append(('clip_rmsprop', ev()))
        with torch.no_grad():
            T = tr.T
            for nm in ('idx', 'val', 'count'):
                getattr(tr.pobs, nm)[0].copy_(getattr(tr.pobs, nm)[T])
            tr.act_in[0].copy_(tr.act_in[T])
            tr.h0a.copy_(tr.ha)
            tr.h0c.copy_(tr.hc)
            tr.pobs.set_projection(tr.net.obs_proj.weight, tr.net.obs_proj.bias)
            tr.pobs.emb[0].copy_(M._project_dense(tr.pobs.idx[0], tr.pobs.val[0], tr.net.obs_proj))
        marks.append(('slide', ev()))
        tr.t = 0
        torch.cuda.synchronize()
        for (_, a), (name, b) in zip(marks, marks[1:]):
            acc[name] = acc.get(name, 0.0) + a.elapsed_time(b) / args.updates
    print(json.dumps({"what": "device ms per A2C update by phase", "config": args.config, "envs": args.batch,
                      "phases_ms": {k: round(v, 3) for k, v in acc.items()},
                      "total_ms": round(sum(acc.values()), 3)}))
    f.close()


if __name__ == '__main__':
    main()

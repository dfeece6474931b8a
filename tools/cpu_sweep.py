#!/usr/bin/env python3
"""How many host cores the CPU baseline can use on this box: the C restatement (bench.cpu_baseline, one env per
process) at several worker counts, a few seconds each, plus the scheduler's view (affinity, cgroup cpu.max).
usage: python tools/cpu_sweep.py [SECONDS] [WORKERS ...] > profiles/<tag>_cpu_sweep.json"""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 4.0
    counts = [int(a) for a in sys.argv[2:]] or [1, 8, 16, 32, 64]
    try:
        cpu_max = Path('/sys/fs/cgroup/cpu.max').read_text().strip()
    except OSError:
        cpu_max = None
    rows = []
    for w in counts:
        v, n, wall = bench.cpu_baseline('large8.yaml', secs, w, 12345)
        rows.append({"workers": w, "env_steps_per_s": round(v, 1), "per_worker": round(v / w, 1), "steps": n,
                     "wall_s": round(wall, 2)})
        print(json.dumps(rows[-1]), file=sys.stderr, flush=True)
    print(json.dumps({"what": "C restatement (oracle/mfg_oracle.c) on large8, 1 env per process, aggregate "
                              "env-steps/s by worker count", "affinity_cores": len(os.sched_getaffinity(0)),
                      "cpu_count": os.cpu_count(), "cgroup_cpu_max": cpu_max, "cpu_model": bench.cpu_model(),
                      "seconds_per_point": secs, "rows": rows}, indent=1))


if __name__ == '__main__':
    main()

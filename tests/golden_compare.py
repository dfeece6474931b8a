"""Replay a reference golden fixture (tests/golden/<tag>_s<seed>.json/.npz) through a stepper and
compare every recorded quantity. Used by the parity tests (oracle vs fixtures, HIP engine vs fixtures)."""
import gzip
import hashlib
import json
from pathlib import Path

import numpy as np

GOLDEN = Path(__file__).resolve().parent / 'golden'


def sha(b):
    return hashlib.sha1(b).hexdigest()[:16]


def load(tag, seed):
    with gzip.open(GOLDEN / f'{tag}_s{seed}.json.gz', 'rt') as f:
        rec = json.load(f)
    npz = np.load(GOLDEN / f'{tag}_s{seed}.npz')
    return rec, npz


def stack_obs(obs_list):
    return np.stack([np.asarray(x, dtype=np.float64) for x in obs_list])


def info_equal(a, b):
    if set(a) != set(b):
        return False, sorted(set(a) ^ set(b))
    bad = [k for k in a if float(a[k]) != float(b[k])]
    return not bad, bad


def posdict_sha(pd):
    return sha(json.dumps(sorted((int(k), v) for k, v in pd.items())).encode())

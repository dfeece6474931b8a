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
    """Per-agent obs (L_a, d, d) f64 -> one array padded with zeros to the largest L (agents may differ)."""
    xs = [np.asarray(x, dtype=np.float64) for x in obs_list]
    lmax = max(x.shape[0] for x in xs)
    out = np.zeros((len(xs), lmax) + xs[0].shape[1:], np.float64)
    for a, x in enumerate(xs):
        out[a, :x.shape[0]] = x
    return out


def obs_bytes(obs_list):
    """Bytes hashed into a fixture's obs_sha: the agents' (L_a, d, d) f64 arrays concatenated in order
    (for equal L this equals np.stack(...).tobytes())."""
    return b''.join(np.ascontiguousarray(x, dtype=np.float64).tobytes() for x in obs_list)


def info_equal(a, b):
    if set(a) != set(b):
        return False, sorted(set(a) ^ set(b))
    bad = [k for k in a if float(a[k]) != float(b[k])]
    return not bad, bad


def posdict_sha(pd):
    return sha(json.dumps(sorted((int(k), v) for k, v in pd.items())).encode())

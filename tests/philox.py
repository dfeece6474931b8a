"""numpy Philox4x32-10 matching csrc/mfg_engine.hip philox_u32 (synthetic actions). Test/baseline helper."""
import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)


def philox_u32(k0, k1, c0, c1):
    k0 = np.asarray(k0, np.uint32).copy(); k1 = np.asarray(k1, np.uint32).copy()
    c0 = np.asarray(c0, np.uint32).copy(); c1 = np.asarray(c1, np.uint32).copy()
    k0, k1, c0, c1 = np.broadcast_arrays(k0, k1, c0, c1)
    k0 = k0.copy(); k1 = k1.copy(); c0 = c0.copy(); c1 = c1.copy()
    c2 = np.zeros_like(c0); c3 = np.zeros_like(c0)
    with np.errstate(over='ignore'):
        for _ in range(10):
            p0 = M0 * c0.astype(np.uint64)
            p1 = M1 * c2.astype(np.uint64)
            n0 = (p1 >> np.uint64(32)).astype(np.uint32) ^ c1 ^ k0
            n2 = (p0 >> np.uint64(32)).astype(np.uint32) ^ c3 ^ k1
            c1 = p1.astype(np.uint32)
            c3 = p0.astype(np.uint32)
            c0, c2 = n0, n2
            k0 = k0 + W0
            k1 = k1 + W1
    return c0


def synthetic_actions(seed, env_ids, step, n_actions):
    """[len(env_ids), A] int32 actions for rollout step `step` (uniform via Lemire multiply-shift)."""
    env_ids = np.asarray(env_ids, np.uint32)[:, None]
    agents = np.arange(len(n_actions), dtype=np.uint32)[None, :]
    u = philox_u32(np.uint32(seed), env_ids, np.uint32(step), agents).astype(np.uint64)
    return ((u * np.asarray(n_actions, np.uint64)[None, :]) >> np.uint64(32)).astype(np.int32)

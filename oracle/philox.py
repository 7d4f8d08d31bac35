"""Philox4x32-10 in numpy (TEST INFRASTRUCTURE ONLY — see oracle/__init__.py).

Restates the engine's RNG contract (DESIGN.md "RNG streams"): counter
(env, episode, attempt, stream), key (seed_lo, seed_hi), Salmon et al. SC'11 constants.
uniform_below(r, n) = (r * n) >> 32.
"""
import numpy as np

STREAM_GOAL = 0
STREAM_START = 1
STREAM_ACTION = 2
STREAM_POLICY = 3

_M0 = np.uint64(0xD2511F53)
_M1 = np.uint64(0xCD9E8D57)
_W0 = 0x9E3779B9
_W1 = 0xBB67AE85
_MASK = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised over broadcastable uint32-compatible counters; returns 4 uint32 arrays."""
    x = np.asarray(c0, dtype=np.uint64) & _MASK
    y = np.asarray(c1, dtype=np.uint64) & _MASK
    z = np.asarray(c2, dtype=np.uint64) & _MASK
    w = np.asarray(c3, dtype=np.uint64) & _MASK
    x, y, z, w = np.broadcast_arrays(x, y, z, w)
    k0 = int(k0) & 0xFFFFFFFF
    k1 = int(k1) & 0xFFFFFFFF
    for _ in range(10):
        p0 = _M0 * x
        p1 = _M1 * z
        hi0, lo0 = p0 >> np.uint64(32), p0 & _MASK
        hi1, lo1 = p1 >> np.uint64(32), p1 & _MASK
        x, y, z, w = (hi1 ^ y ^ np.uint64(k0)), lo1, (hi0 ^ w ^ np.uint64(k1)), lo0
        k0 = (k0 + _W0) & 0xFFFFFFFF
        k1 = (k1 + _W1) & 0xFFFFFFFF
    return (x.astype(np.uint32), y.astype(np.uint32), z.astype(np.uint32), w.astype(np.uint32))


def uniform_below(r, n):
    return ((np.asarray(r, dtype=np.uint64) * np.uint64(n)) >> np.uint64(32)).astype(np.int64)


def seed_key(seed):
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    return seed & 0xFFFFFFFF, seed >> 32

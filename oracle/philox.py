"""Philox4x32-10 (Random123) and the synthetic random policy, in numpy.

TEST INFRASTRUCTURE ONLY.  The policy is the benchmark's action source for
BASELINE config 2 (no reference counterpart: the reference samples actions
with np.random.choice, block_blast_env.py:318-323); it must match the kernel's
``random_policy`` (csrc/bb_device.h) bit for bit.
"""
from __future__ import annotations

import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(idx, step, seed):
    """Vectorised over idx (u64 array); returns 4 uint32 arrays."""
    idx = np.asarray(idx, dtype=np.uint64)
    step = np.uint64(step)
    c0 = idx & MASK32
    c1 = idx >> np.uint64(32)
    c2 = np.full_like(idx, step & MASK32)
    c3 = np.full_like(idx, step >> np.uint64(32))
    k0 = int(seed) & 0xFFFFFFFF
    k1 = (int(seed) >> 32) & 0xFFFFFFFF
    for r in range(10):
        if r:
            k0 = (k0 + W0) & 0xFFFFFFFF
            k1 = (k1 + W1) & 0xFFFFFFFF
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK32
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK32
        c0, c1, c2, c3 = hi1 ^ c1 ^ np.uint64(k0), lo1, hi0 ^ c3 ^ np.uint64(k1), lo0
    return [x.astype(np.uint32) for x in (c0, c1, c2, c3)]


def random_policy(mask_bool: np.ndarray, seed: int, step: int, env_offset: int = 0) -> np.ndarray:
    """mask_bool (N, 192) -> int32 actions: the k-th legal action with
    k = (philox word0 * popcount) >> 32 (0 when no action is legal)."""
    n = mask_bool.shape[0]
    w0 = philox4x32_10(np.arange(n, dtype=np.uint64) + np.uint64(env_offset), step, seed)[0].astype(np.uint64)
    cnt = mask_bool.sum(axis=1).astype(np.uint64)
    k = (w0 * cnt) >> np.uint64(32)
    out = np.zeros(n, dtype=np.int32)
    for i in range(n):
        if cnt[i]:
            out[i] = np.nonzero(mask_bool[i])[0][int(k[i])]
    return out


def sample_uniform(n: int, seed: int, step: int, env_offset: int = 0) -> np.ndarray:
    """The masked-sample kernel's default uniform: philox word1 * 2^-32 (f64)."""
    w1 = philox4x32_10(np.arange(n, dtype=np.uint64) + np.uint64(env_offset), step, seed)[1]
    return w1.astype(np.float64) * 2.0 ** -32

"""Per-epoch record shuffling of the resident training set: the host twin of csrc/feed.h (bit-exact).

The reference's Trainer reads its training files with `read_batch_features(..., randomize_input=True)`
(`airflow-dags/taxi_utils.py:275-276`), a new random order every epoch. The fused GPU trainers keep the records
resident and evaluate a per-epoch pseudo-random permutation of [0, n) per record inside the kernel's fetch; the
CPU trainer and the tests use these functions to compute the same record indices:

    p = step * gstride + goff + row;  e = p // n;  i = p % n
    record = i                                               (seed 0: stored order)
             4 feistel_perm(i // 4, n // 4, epoch_key(seed, e)) + i % 4     (otherwise; i < 4 (n // 4))
             i                                               (the n % 4 records past the last whole group)

The shuffle permutes GROUPS of GROUP = 4 consecutive records (one 128-byte line of 32-byte records) -- see
csrc/feed.h. feistel_perm is a bijection of [0, m) for every m >= 1 and key: a 4-round balanced Feistel network on
[0, 4^h) (4^h >= m) with cycle walking."""
from __future__ import annotations

import numpy as np

_M32 = np.uint64(0xFFFFFFFF)
GROUP_LOG2 = 2  # csrc/feed.h MIFX_SHUFFLE_GLOG2
GROUP = 1 << GROUP_LOG2


def _mix32(x: np.ndarray) -> np.ndarray:
    """lowbias32 on uint64 arrays holding 32-bit values."""
    x = x & _M32
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & _M32
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & _M32
    x ^= x >> np.uint64(16)
    return x


def _mix32_int(x: int) -> int:
    return int(_mix32(np.array([x & 0xFFFFFFFF], dtype=np.uint64))[0])


def epoch_key(key: int, epoch: int) -> int:
    a = _mix32_int((key & 0xFFFFFFFF) ^ _mix32_int(((epoch & 0xFFFFFFFF) + 0x9E3779B9) & 0xFFFFFFFF))
    b = _mix32_int(((key >> 32) & 0xFFFFFFFF) ^ _mix32_int((((epoch >> 32) & 0xFFFFFFFF) + 0x85EBCA6B) & 0xFFFFFFFF)
                   ^ a)
    return (b << 32) | a


def feistel_half(n: int) -> int:
    h = 1
    while h < 32 and (1 << (2 * h)) < n:
        h += 1
    return h


def feistel_perm(i: np.ndarray, n: int, ekey: int, h: int | None = None) -> np.ndarray:
    """The permuted index of every entry of `i` (int array, values in [0, n))."""
    h = feistel_half(n) if h is None else h
    mask = np.uint64((1 << h) - 1)
    k0, k1 = ekey & 0xFFFFFFFF, (ekey >> 32) & 0xFFFFFFFF
    rk = [np.uint64(k) for k in (k0, k1, k0 ^ 0x68E31DA4, k1 ^ 0xB5297A4D)]
    sh = np.uint64(h)
    x = np.asarray(i, dtype=np.uint64).copy()
    todo = np.ones(x.shape, dtype=bool)  # every index walks at least once
    while todo.any():
        v = x[todo]
        L, R = v >> sh, v & mask
        for r in range(4):
            t = L ^ (_mix32((R & _M32) ^ rk[r] ^ (R >> np.uint64(32))) & mask)
            L, R = R, t
        x[todo] = (L << sh) | R
        todo[todo] = x[todo] >= np.uint64(n)
    return x.astype(np.int64)


def record_indices(step: int, batch: int, n: int, gstride: int | None = None, goff: int = 0,
                   seed: int = 0) -> np.ndarray:
    """Records of the `batch` rows one replica trains on at `step` (see module docstring)."""
    gstride = batch if gstride is None else gstride
    if not (0 < batch <= n and gstride >= batch and 0 <= goff and goff + batch <= gstride):
        raise ValueError("need 0 < batch <= n and goff + batch <= gstride")
    p0 = step * gstride + goff
    e0, i0 = divmod(p0, n)
    i = i0 + np.arange(batch, dtype=np.int64)
    e = np.full(batch, e0, dtype=np.int64)
    wrap = i >= n
    i[wrap] -= n
    e[wrap] += 1
    if seed == 0:
        return i
    ng = n >> GROUP_LOG2
    out = i.copy()  # records past the last whole group keep their place
    h = feistel_half(max(ng, 1))
    for ep in np.unique(e):
        sel = (e == ep) & (i < ng * GROUP)
        if sel.any():
            g = feistel_perm(i[sel] >> GROUP_LOG2, ng, epoch_key(int(seed), int(ep)), h)
            out[sel] = (g << GROUP_LOG2) | (i[sel] & (GROUP - 1))
    return out

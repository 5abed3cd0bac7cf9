"""torch.randperm(n, generator=torch.Generator().manual_seed(s)) on the device.

``DistributedSampler`` (the reference's sampler, ddp_gpus.py:72-79; torch
utils/data/distributed.py) draws each epoch's order as
``torch.randperm(len(ds), generator=g.manual_seed(seed + epoch))`` on the CPU:
an mt19937 stream and a sequential Fisher-Yates pass,

    r = arange(n); for i in 0..n-2: z = mt() % (n - i); swap(r[i], r[i + z]).

That is ~20 us of host time per epoch, longer than a whole W=8 epoch of the
persistent engine. ``csrc/kernels/torch_perm.hip`` computes the identical
permutation on the GPU, one workgroup per epoch, without the sequential pass:

* mt19937 seeding (623 dependent steps, one lane), then each 624-word twist in
  three parallel phases (words [0,227) read only old words, [227,454) read
  phase-1 words, [454,624) phase-2 words), tempering elementwise;
* t_i = i + (mt_i mod (n - i)) for all i in parallel;
* the swap sequence resolved in parallel. Position i is final after step i and
  receives what position t_i held just before step i. Position p (> k) only
  changes at steps k with t_k = p, taking what position k held before step k.
  With C(k) = max{j < k : t_j = k} and A(i) = max{j < i : t_j = t_i}:
      B[k] = B[C(k)] if C(k) exists else k      (value at k before step k)
      perm[i] = B[A(i)] if A(i) exists else t_i,  perm[n-1] = B[n-1].

This module is the host model of that kernel (numpy, same algorithm) used by
the CPU tests to pin the algorithm against ``torch.randperm`` itself.
"""
from __future__ import annotations

import numpy as np

N_MT, M_MT = 624, 397
MATRIX_A, UPPER, LOWER = 0x9908B0DF, 0x80000000, 0x7FFFFFFF


def mt19937_init(seed: int) -> np.ndarray:
    """torch CPUGeneratorImpl.manual_seed(seed): mt19937 init_with_uint32(seed)."""
    st = np.zeros(N_MT, dtype=np.uint64)
    st[0] = seed & 0xFFFFFFFF
    for j in range(1, N_MT):
        prev = int(st[j - 1])
        st[j] = (1812433253 * (prev ^ (prev >> 30)) + j) & 0xFFFFFFFF
    return st.astype(np.uint32)


def mt19937_twist(st: np.ndarray) -> np.ndarray:
    """One next_state() in the kernel's three parallel phases."""
    s = st.astype(np.uint64).copy()

    def tw(u, v):
        y = (u & UPPER) | (v & LOWER)
        return (y >> 1) ^ np.where((v & 1) != 0, MATRIX_A, 0).astype(np.uint64)

    k = N_MT - M_MT  # 227
    i1 = np.arange(0, k)
    new = s.copy()
    new[i1] = s[i1 + M_MT] ^ tw(s[i1], s[i1 + 1])
    i2 = np.arange(k, 2 * k)
    new[i2] = new[i2 - k] ^ tw(s[i2], s[i2 + 1])
    i3 = np.arange(2 * k, N_MT - 1)
    new[i3] = new[i3 - k] ^ tw(s[i3], s[i3 + 1])
    new[N_MT - 1] = new[N_MT - 1 - k] ^ tw(s[N_MT - 1:N_MT], new[0:1])[0]
    return new.astype(np.uint32)


def temper(y: np.ndarray) -> np.ndarray:
    y = y.astype(np.uint64)
    y ^= y >> 11
    y ^= (y << 7) & 0x9D2C5680
    y ^= (y << 15) & 0xEFC60000
    y ^= y >> 18
    return (y & 0xFFFFFFFF).astype(np.uint32)


def mt19937_stream(seed: int, count: int) -> np.ndarray:
    st = mt19937_init(seed)
    out = []
    while sum(len(o) for o in out) < count:
        st = mt19937_twist(st)
        out.append(temper(st))
    return np.concatenate(out)[:count] if out else np.zeros(0, np.uint32)


def randperm(n: int, seed: int) -> np.ndarray:
    """== torch.randperm(n, generator=torch.Generator().manual_seed(seed)).numpy()."""
    if n <= 1:
        return np.arange(n, dtype=np.int64)
    r = mt19937_stream(seed, n - 1).astype(np.int64)
    i = np.arange(n - 1, dtype=np.int64)
    t = i + r % (n - i)
    # C(k) = last writer of position k before step k (writers with t_j > j only)
    C = np.full(n, -1, dtype=np.int64)
    mv = t > i
    np.maximum.at(C, t[mv], i[mv])
    # A(i) = previous writer (in step order) of the same target
    A = np.full(n - 1, -1, dtype=np.int64)
    order = np.lexsort((i, t))
    ts, js = t[order], i[order]
    same = np.concatenate([[False], ts[1:] == ts[:-1]])
    A[js[same]] = js[np.nonzero(same)[0] - 1]
    A = np.where(t == i, C[:n - 1], A)
    B = np.arange(n, dtype=np.int64)  # chains run to smaller indices: resolve in order
    for k in range(n):
        if C[k] >= 0:
            B[k] = B[C[k]]
    perm = np.empty(n, dtype=np.int64)
    perm[:n - 1] = np.where(A >= 0, B[np.maximum(A, 0)], t)
    perm[n - 1] = B[n - 1]
    return perm


def rank_indices(n: int, seed: int, epoch: int, world: int, rank: int, shuffle: bool = True,
                 drop_last: bool = False) -> np.ndarray:
    """DistributedSampler(ds of n, world, rank, shuffle, seed, drop_last) indices of ``epoch``."""
    perm = randperm(n, seed + epoch) if shuffle else np.arange(n)
    if drop_last and n % world:
        num = n // world
    else:
        num = -(-n // world)
    q = rank + world * np.arange(num)
    return perm[q % n]

"""numpy twin of gen_records64_kernel (csrc/kernels/generators.hip): the 64-byte record store
``gen://records64`` used by the GroupBy-Aggregate and hash-join benchmarks."""
from __future__ import annotations

import numpy as np

from .terasort_cpu import mix64

G = np.uint64(0x9E3779B97F4A7C15)
H = np.uint64(0xD1B54A32D192ED03)
FIELDS = ["Key"] + [f"V{j}" for j in range(1, 8)]


def dim_multiplier(nkeys: int) -> int:
    """An odd multiplier coprime with nkeys (makes i -> (i*A + seed) % nkeys a bijection)."""
    import math
    a = 0x9E3779B1 % max(nkeys, 2) | 1
    while math.gcd(a, nkeys) != 1:
        a += 2
    return a


def gen_columns(first: int, n: int, nkeys: int, seed: int, ncols: int = 8, dim_mult: int = 0) -> list:
    i = np.arange(first, first + n, dtype=np.uint64)
    s = np.uint64(seed & (2**64 - 1))
    if dim_mult:
        key = np.array([(int(x) * dim_mult + (seed & (2**64 - 1))) % nkeys for x in i], dtype=np.uint64)
        with np.errstate(over="ignore"):
            cols = [key.astype(np.int64)]
            for j in range(1, ncols):
                cols.append((mix64((s + np.uint64(j) * H) ^ key) >> np.uint64(33)).astype(np.int64))
        return cols
    with np.errstate(over="ignore"):
        cols = [(mix64(s ^ (i * G)) % np.uint64(nkeys)).astype(np.int64)]
        for j in range(1, ncols):
            cols.append((mix64((s + np.uint64(j) * H) ^ i) >> np.uint64(33)).astype(np.int64))
    return cols


def gen_records(first: int, n: int, nkeys: int, seed: int, ncols: int = 8, dim_mult: int = 0) -> list:
    cols = gen_columns(first, n, nkeys, seed, ncols, dim_mult)
    return list(zip(*[c.tolist() for c in cols]))

"""Host (numpy) implementation of the synthetic TeraSort record generator.

Bit-exact twin of ``ts_record`` in csrc/kernels/terasort.hip: used by the object executor (CPU
workers reading ``gen://terasort``) and as the reference the GPU generator is tested against.
"""
from __future__ import annotations

import numpy as np

M1 = np.uint64(0x9E3779B97F4A7C15)
M2 = np.uint64(0xBF58476D1CE4E5B9)
M3 = np.uint64(0x94D049BB133111EB)


def mix64(z: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = (z + M1).astype(np.uint64)
        z = ((z ^ (z >> np.uint64(30))) * M2).astype(np.uint64)
        z = ((z ^ (z >> np.uint64(27))) * M3).astype(np.uint64)
        return z ^ (z >> np.uint64(31))


def gen_array(first: int, n: int, seed: int) -> np.ndarray:
    """Records first..first+n-1 as a uint8 array [n, 100]."""
    g = np.arange(first, first + n, dtype=np.uint64)
    s = np.uint64(seed & (2**64 - 1))
    with np.errstate(over="ignore"):
        kA = mix64(s ^ mix64(g))
        kB = mix64(kA ^ np.uint64(0xD1B54A32D192ED03))
        fil = mix64(g ^ (s * np.uint64(0x2545F4914F6CDD1D)).astype(np.uint64) ^ np.uint64(0xF00DF00DF00DF00D))
    out = np.empty((n, 100), dtype=np.uint8)
    for b in range(8):
        out[:, b] = ((kA >> np.uint64(56 - 8 * b)) & np.uint64(0xFF)).astype(np.uint8)
    out[:, 8] = ((kB >> np.uint64(56)) & np.uint64(0xFF)).astype(np.uint8)
    out[:, 9] = ((kB >> np.uint64(48)) & np.uint64(0xFF)).astype(np.uint8)
    out[:, 10] = 0x00
    out[:, 11] = 0x11
    out[:, 12:28] = ord("0")
    hexd = np.frombuffer(b"0123456789ABCDEF", dtype=np.uint8)
    for q in range(16, 32):
        nib = ((g >> np.uint64(4 * (31 - q))) & np.uint64(0xF)).astype(np.int64)
        out[:, 12 + q] = hexd[nib]
    out[:, 44:48] = np.array([0x88, 0x99, 0xAA, 0xBB], dtype=np.uint8)
    for i in range(12):
        letter = (ord("A") + ((fil >> np.uint64(5 * i)) % np.uint64(26))).astype(np.uint8)
        out[:, 48 + 4 * i: 52 + 4 * i] = letter[:, None]
    out[:, 96:100] = np.array([0xCC, 0xDD, 0xEE, 0xFF], dtype=np.uint8)
    return out


def gen_records(first: int, n: int, seed: int) -> list:
    a = gen_array(first, n, seed)
    return [bytes(r) for r in a]


def record_hash(rows: np.ndarray) -> np.ndarray:
    """FNV-1a over the 25 little-endian dwords, then mix64 (matches rec_hash in the kernel)."""
    w = rows.reshape(-1, 100).view("<u4").astype(np.uint64)
    h = np.full(w.shape[0], 0xCBF29CE484222325, dtype=np.uint64)
    with np.errstate(over="ignore"):
        for k in range(25):
            h = ((h ^ w[:, k]) * np.uint64(0x100000001B3)).astype(np.uint64)
    return mix64(h)


def checksum(rows: np.ndarray) -> int:
    with np.errstate(over="ignore"):
        return int(record_hash(rows).sum(dtype=np.uint64))

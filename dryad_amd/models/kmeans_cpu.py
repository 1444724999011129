"""Host (numpy) twin of the k-means point generator (``kmeans_gen_kernel`` in
csrc/kernels/kmeans.hip) and a float64 reference step, used by the object/CPU executors reading
``gen://points`` and by tests."""
from __future__ import annotations

import numpy as np

from .terasort_cpu import mix64

DIM = 128


def _u01(z: np.ndarray) -> np.ndarray:
    return (mix64(z) >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0)


def gen_points(first: int, n: int, blobs: int, seed: int, dim: int = DIM) -> np.ndarray:
    """Points first..first+n-1 as float32 [n, dim] (bit-identical to the GPU generator)."""
    if dim != DIM:
        raise ValueError("the point generator is defined for dim=128")
    i = np.arange(first, first + n, dtype=np.uint64)[:, None]
    d = np.arange(dim, dtype=np.uint64)[None, :]
    s = np.uint64(seed & (2**64 - 1))
    with np.errstate(over="ignore"):
        b = (i * np.uint64(2654435761)) % np.uint64(blobs)
        zc = s ^ (b * np.uint64(0x9E3779B97F4A7C15)) ^ (d * np.uint64(0x632BE59BD9B4E019))
        zn = s * np.uint64(31) + i * np.uint64(0xD1B54A32D192ED03) + d
    centre = np.float32(10.0) * _u01(zc) - np.float32(5.0)
    noise = _u01(zn) - np.float32(0.5)
    return (centre + np.float32(0.2) * noise).astype(np.float32)


def gen_point_records(first: int, n: int, blobs: int, seed: int) -> list:
    return [tuple(r) for r in gen_points(first, n, blobs, seed).tolist()]


def step_reference(points: np.ndarray, centroids: np.ndarray):
    """(sums f64 [K, D], counts i64 [K]) of one assignment step, float64 distances."""
    x = points.astype(np.float64)
    c = centroids.astype(np.float64)
    d = (c * c).sum(1)[None, :] - 2.0 * x @ c.T
    a = np.argmin(d, axis=1)
    k = c.shape[0]
    sums = np.zeros((k, x.shape[1]))
    np.add.at(sums, a, x)
    return sums, np.bincount(a, minlength=k)

"""k-means step on MFMA (HIP kernels in csrc/kernels/kmeans.hip).

BASELINE config: "k-means on 1B x 128-dim points (Apply/Fork iterative DAG, MFMA reductions)".
The reference runs k-means as a DoWhile over per-partition Apply bodies that compute nearest
centroids and partial sums on the CPU, then a final aggregation stage (reference samples under
DryadLinq/Samples and DryadLinqTests iterative jobs).  Here one kernel per partition does the
assignment (f32 MFMA distance tiles + argmin) and the LDS-privatised partial sums; the cross-rank
reduction is one RCCL all-reduce of K*(D+1) values.
"""
from __future__ import annotations

import torch

from . import _lib
from ._lib import c_i32, c_u64, ptr, stream_of, vp

DIM = 128

_lib.register_signatures({
    "dr_kmeans_mode": (c_i32, [c_i32]),
    "dr_kmeans_step": (c_i32, [vp, c_u64, c_i32, vp, c_i32, vp, vp, vp, vp, vp, vp]),
    "dr_kmeans_near_workspace": (c_u64, [c_u64]),
    "dr_kmeans_gen": (c_i32, [vp, c_u64, c_i32, c_u64, c_i32, c_u64, vp]),
})


class KMeansWorkspace:
    """Per-K scratch buffers reused across iterations (no allocation inside the loop)."""

    def __init__(self, n: int, k: int, device):
        self.k = k
        self.cnorm = torch.empty(k, dtype=torch.float32, device=device)
        self.assign = torch.empty(n, dtype=torch.int32, device=device)
        self.sums = torch.empty((k, DIM), dtype=torch.float64, device=device)
        self.counts = torch.empty(k, dtype=torch.int64, device=device)
        # near-tie list of the K <= 64 bf16-MFMA path (count + (point, estimate) pairs)
        self.near = torch.empty(int(_lib.lib().dr_kmeans_near_workspace(c_u64(n))) if k <= 64 else 16,
                                dtype=torch.uint8, device=device)


def mode(k: int) -> int:
    """0: centroids + accumulator slab in LDS; 1: streamed centroid tiles + slab; 2: two-pass;
    3: K <= 64 on bf16 MFMA (split-precision distances, exact re-rank of near ties, MFMA sums)."""
    return int(_lib.lib().dr_kmeans_mode(k))


def generate(points: torch.Tensor, first: int = 0, blobs: int = 64, seed: int = 0x6B6D) -> torch.Tensor:
    """Deterministic synthetic Gaussian-blob points (counter based: slices of a global set agree)."""
    _lib.require_gpu_tensor(points, "kmeans.generate")
    assert points.dtype == torch.float32 and points.dim() == 2 and points.shape[1] == DIM
    _lib.call("dr_kmeans_gen", ptr(points), c_u64(points.shape[0]), DIM, c_u64(first), int(blobs),
              c_u64(seed), stream_of(points))
    return points


def step(points: torch.Tensor, centroids: torch.Tensor, ws: KMeansWorkspace | None = None):
    """One assignment + partial-sum pass.  Returns (sums f64 [K,D], counts i64 [K], assign i32 [n])."""
    _lib.require_gpu_tensor(points, "kmeans.step")
    _lib.require_gpu_tensor(centroids, "kmeans.step")
    assert points.dtype == torch.float32 and centroids.dtype == torch.float32
    assert points.shape[1] == DIM and centroids.shape[1] == DIM
    n, k = points.shape[0], centroids.shape[0]
    if ws is None or ws.k != k or ws.assign.shape[0] < n:
        ws = KMeansWorkspace(n, k, points.device)
    ws.sums.zero_()
    ws.counts.zero_()
    _lib.call("dr_kmeans_step", ptr(points), c_u64(n), DIM, ptr(centroids), k, ptr(ws.cnorm), ptr(ws.assign),
              ptr(ws.sums), ptr(ws.counts), ptr(ws.near), stream_of(points))
    return ws.sums, ws.counts, ws.assign[:n]


def update(centroids: torch.Tensor, sums: torch.Tensor, counts: torch.Tensor) -> torch.Tensor:
    """New centroids = sums / counts; empty clusters keep their old centre."""
    c = counts.to(torch.float64).unsqueeze(1)
    new = torch.where(c > 0, sums / c.clamp_min(1), centroids.to(torch.float64))
    return new.to(torch.float32)


def step_reference(points: torch.Tensor, centroids: torch.Tensor):
    """Plain PyTorch fp32 reference of the same op (for numerics tests)."""
    d = (centroids * centroids).sum(1)[None, :] - 2.0 * points @ centroids.T
    a = torch.argmin(d, dim=1)
    k = centroids.shape[0]
    sums = torch.zeros((k, DIM), dtype=torch.float64, device=points.device)
    sums.index_add_(0, a, points.to(torch.float64))
    counts = torch.bincount(a, minlength=k)
    return sums, counts, a.to(torch.int32), d

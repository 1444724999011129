"""k-means step on MFMA (HIP kernels in csrc/kernels/kmeans.hip).

K <= 64 (the benchmark's K = 64) runs on a per-table state (``SplitPoints``, cached per point
tensor): the bf16 rounding of every coordinate and |x| per point, written once, so an
iteration's assignment kernel reads half the bytes of the f32 rows; and the per-cluster sums and
counts, kept with the table and updated only for the points whose cluster changed (their exact
f32 rows move from the old cluster's sums to the new one's).  Larger K, or a plane that does not
fit in free HBM, use the f32 kernels.
"""
from __future__ import annotations

import weakref

import torch

from . import _lib
from ._lib import c_i32, c_u64, ptr, stream_of, vp

DIM = 128

_lib.register_signatures({
    "dr_kmeans_mode": (c_i32, [c_i32]),
    "dr_kmeans_step": (c_i32, [vp, c_u64, c_i32, vp, c_i32, vp, vp, vp, vp, vp, vp]),
    "dr_kmeans_near_workspace": (c_u64, [c_u64]),
    "dr_kmeans_gen": (c_i32, [vp, c_u64, c_i32, c_u64, c_i32, c_u64, vp]),
    "dr_kmeans_hi": (c_i32, [vp, c_u64, vp, vp, vp]),
    "dr_kmeans_step_hi": (c_i32, [vp, vp, vp, c_u64, vp, c_i32, vp, vp, vp, vp, vp, vp, vp]),
})

PLANES_MAX_K = 64
# free HBM kept beyond the planes (the step's workspace and whatever the job allocates next)
PLANES_HEADROOM = 4 << 30


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


class SplitPoints:
    """Per-point-table state of the K <= 64 path: ``xh`` [n, 128] bf16 (round-to-nearest of x),
    ``xnorm`` |x| per point, and the running per-cluster state of the last step: ``prev`` (final
    assignment, -1 = none), ``sums`` (K x 128 f64) and ``counts`` (K i64)."""

    def __init__(self, x: torch.Tensor):
        n = x.shape[0]
        self.n = n
        self.version = x._version
        self.xh = torch.empty((n, DIM), dtype=torch.bfloat16, device=x.device)
        self.xnorm = torch.empty(n, dtype=torch.float32, device=x.device)
        self.prev = torch.full((n,), -1, dtype=torch.int32, device=x.device)
        self.sums = self.counts = None
        if x.is_cuda:
            _lib.call("dr_kmeans_hi", ptr(x), c_u64(n), ptr(self.xh), ptr(self.xnorm), stream_of(x))
        else:
            self.xh.copy_(x.bfloat16())
            self.xnorm.copy_(x.double().norm(dim=1).float())

    def state_for(self, k: int):
        """The running sums / counts for ``k`` clusters; a new K restarts them (every point moves)."""
        if self.sums is None or self.sums.shape[0] != k:
            self.sums = torch.zeros((k, DIM), dtype=torch.float64, device=self.xh.device)
            self.counts = torch.zeros(k, dtype=torch.int64, device=self.xh.device)
            self.prev.fill_(-1)
        return self.sums, self.counts


# (device, data_ptr, n) -> SplitPoints.  The entry lives as long as the tensor that owns the
# points' memory (the base of whatever view the caller passes: a table column handed out as a new
# view every iteration still hits), and is checked against that owner and its version counter.
_SPLITS: dict = {}


def split_bytes(n: int) -> int:
    return n * (DIM * 2 + 4 + 4)


def split_points(x: torch.Tensor, create: bool = True) -> SplitPoints | None:
    """The cached split of ``x`` (recomputed if ``x`` was modified in place since).  Returns None
    when the planes do not fit in free HBM (the caller then runs the f32 kernels)."""
    base = x if x._base is None else x._base
    key = (str(x.device), x.data_ptr(), x.shape[0])
    sp = _SPLITS.get(key)
    if sp is not None and sp.owner() is base and sp.version == x._version:
        return sp
    if not create:
        return None
    _SPLITS.pop(key, None)
    if x.is_cuda:
        free, _total = torch.cuda.mem_get_info(x.device)
        cached = torch.cuda.memory_reserved(x.device) - torch.cuda.memory_allocated(x.device)
        if split_bytes(x.shape[0]) + PLANES_HEADROOM > free + cached:
            return None
    sp = SplitPoints(x)

    def _drop(ref, key=key):
        cur = _SPLITS.get(key)
        if cur is not None and cur.owner is ref:
            del _SPLITS[key]

    sp.owner = weakref.ref(base, _drop)
    _SPLITS[key] = sp
    return sp


def split_reference(x: torch.Tensor):
    """torch twin of kmeans_split_kernel: x = xh + xm + xl, each a round-to-nearest bf16 of the
    remainder so far (exact: the remainders are exact in f32 and 3 x 8 significand bits cover 24;
    for |x| >= 2^-100, where the remainders stay normal numbers)."""
    x = x.float()
    h = x.bfloat16()
    r1 = x - h.float()
    m = r1.bfloat16()
    lo = (r1 - m.float()).bfloat16()
    return h, m, lo


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
    _lib.written(points)
    return points


def step(points: torch.Tensor, centroids: torch.Tensor, ws: KMeansWorkspace | None = None,
         planes: bool | None = None):
    """One assignment + partial-sum pass.  Returns (sums f64 [K,D], counts i64 [K], assign i32 [n]).

    ``planes``: None = the bf16-plane path with kept sums when K <= 64 and the plane fits (the
    default), False = the f32 kernels, True = the plane path or an error."""
    _lib.require_gpu_tensor(points, "kmeans.step")
    _lib.require_gpu_tensor(centroids, "kmeans.step")
    assert points.dtype == torch.float32 and centroids.dtype == torch.float32
    assert points.shape[1] == DIM and centroids.shape[1] == DIM
    n, k = points.shape[0], centroids.shape[0]
    if ws is None or ws.k != k or ws.assign.shape[0] < n:
        ws = KMeansWorkspace(n, k, points.device)
    ws.sums.zero_()
    ws.counts.zero_()
    sp = None
    if planes is not False and 1 <= k <= PLANES_MAX_K and n > 0:
        sp = split_points(points)
        if sp is None and planes:
            raise MemoryError(f"kmeans.step: the bf16 plane of {n} points ({split_bytes(n) >> 20} MiB) does not fit")
    elif planes:
        raise ValueError(f"kmeans.step: the plane path needs 1 <= K <= {PLANES_MAX_K} (K = {k})")
    if sp is not None:
        sums, counts = sp.state_for(k)
        _lib.call("dr_kmeans_step_hi", ptr(sp.xh), ptr(sp.xnorm), ptr(points), c_u64(n), ptr(centroids), k,
                  ptr(ws.cnorm), ptr(ws.assign), ptr(sp.prev), ptr(sums), ptr(counts), ptr(ws.near),
                  stream_of(points))
        ws.sums.copy_(sums)
        ws.counts.copy_(counts)
        return ws.sums, ws.counts, ws.assign[:n]
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

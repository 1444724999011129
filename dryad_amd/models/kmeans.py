"""k-means as an iterative DryadLINQ job (BASELINE config "k-means on 1B x 128-dim points
(Apply/Fork iterative DAG, MFMA reductions)").

The reference expresses k-means as a client-side ``DoWhile`` (DryadLinqQueryable.cs:1280-1306)
whose body is per-partition ``Apply`` work plus a merge: every iteration is one DryadLINQ job.
Here the same query shape runs on the GPU executor:

    points.ApplyPerPartition(centroids, partial_sums, is_first_only=True)   # broadcast centroids
          .Apply(centroids, combine)                                         # merge to 1 partition

* ``partial_sums`` is a ``@device_function``: on each GPU it is ONE fused HIP kernel over the
  HBM-resident partition (f32 MFMA distance tiles, in-lane argmin, LDS-privatised sums; see
  csrc/kernels/kmeans.hip) returning a K-row table (cluster, count, f64 sums);
* the K-row partials of all partitions are gathered and ``combine`` divides sums by counts;
* the point table is materialised once in HBM (``hbm://``) and re-read by every iteration, so an
  iteration moves only K x 128 centroids plus K partial rows per GPU.

The same functions run under LocalDebug / the CPU executors on CPU-tensor tables (torch), which
is how the GPU result is checked against the oracle in the tests.
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field

import numpy as np
import torch

from .. import types as T
from ..attributes import device_function
from ..gpu.table import DeviceTable, Shape
from .kmeans_cpu import DIM, gen_points

POINT_T = T.Vector(T.Float32, DIM)
_WS: dict = {}


def _step(x: torch.Tensor, c: torch.Tensor):
    """(sums f64 [K, D], counts i64 [K]) for one partition: HIP kernel on the GPU, torch on CPU."""
    if x.is_cuda:
        from ..ops import kmeans as KM
        key = (x.device, c.shape[0])
        ws = _WS.get(key)
        if ws is None or ws.assign.shape[0] < x.shape[0]:
            ws = _WS[key] = KM.KMeansWorkspace(x.shape[0], c.shape[0], x.device)
        sums, counts, _ = KM.step(x, c, ws)
        return sums.clone(), counts.clone()
    xd, cd = x.double(), c.double()
    d = (cd * cd).sum(1)[None, :] - 2.0 * xd @ cd.T
    a = torch.argmin(d, dim=1)
    sums = torch.zeros((c.shape[0], x.shape[1]), dtype=torch.float64).index_add_(0, a, xd)
    return sums, torch.bincount(a, minlength=c.shape[0]).to(torch.int64)


@device_function
def partial_sums(points: DeviceTable, cents: DeviceTable) -> DeviceTable:
    """Per-partition assignment + partial sums (the homomorphic Apply body)."""
    x = points.col(0)
    c = cents.col(0).to(device=x.device, dtype=torch.float32).contiguous()
    k = c.shape[0]
    if points.n == 0:
        sums = torch.zeros((k, x.shape[1]), dtype=torch.float64, device=x.device)
        counts = torch.zeros(k, dtype=torch.int64, device=x.device)
    else:
        sums, counts = _step(x.contiguous(), c)
    ids = torch.arange(k, dtype=torch.int32, device=x.device)
    return DeviceTable.from_columns({"k": ids, "n": counts, "s": sums}, Shape("tuple", ["k", "n", "s"]))


@device_function
def combine(parts: DeviceTable, cents: DeviceTable) -> DeviceTable:
    """Merge the partials of all partitions into the next centroids (empty clusters stay put)."""
    old = cents.col(0)
    dev = old.device
    k = old.shape[0]
    ids = parts.col(0).to(dev).long()
    n = torch.zeros(k, dtype=torch.int64, device=dev).index_add_(0, ids, parts.col(1).to(dev).long())
    s = torch.zeros((k, old.shape[1]), dtype=torch.float64, device=dev).index_add_(
        0, ids, parts.col(2).to(dev).double())
    nd = n.to(torch.float64).unsqueeze(1)
    new = torch.where(nd > 0, s / nd.clamp_min(1), old.double()).to(torch.float32)
    return DeviceTable.from_columns({"x": new}, Shape("vector", ["x"], POINT_T))


def step_query(points, cents):
    """One k-means iteration as a query over the points table and a centroid table."""
    return points.ApplyPerPartition(cents, partial_sums, is_first_only=True).Apply(cents, combine)


@dataclass
class KMeansConfig:
    points_per_partition: int = 125_000_000     # 8 GPUs -> 1e9 points x 128 dims (512 GB f32)
    k: int = 64
    blobs: int = 64
    seed: int = 0x6B6D
    iterations: int = 5
    tol: float = 0.0


@dataclass
class KMeansResult:
    centroids: np.ndarray
    iterations: int
    seconds_per_iteration: list = field(default_factory=list)


class KMeansJob:
    """Driver: materialise points once, iterate ``step_query`` (explicit loop or ``DoWhile``)."""

    def __init__(self, ctx, cfg: KMeansConfig, partitions: int | None = None, materialize: bool = True):
        self.ctx, self.cfg = ctx, cfg
        self.partitions = int(partitions or getattr(ctx, "PartitionCount", 1) or 1)
        n = cfg.points_per_partition * self.partitions
        self.n = n
        self.source_uri = (f"gen://points?count={n}&partitions={self.partitions}&blobs={cfg.blobs}"
                           f"&seed={cfg.seed}")
        pts = ctx.FromStore(self.source_uri)
        if materialize and not getattr(ctx, "LocalDebug", False):
            uri = f"{ctx.StorageScheme}://kmeans_points_{abs(hash(self.source_uri)) % 10**8}" \
                if ctx.StorageScheme == "hbm" else ctx.MakeTemporaryStreamUri()
            pts.ToStore(uri, delete_if_exists=True).SubmitAndWait()
            pts = ctx.FromStore(uri)
        self.points = pts

    def initial_centroids(self) -> list:
        """The first K generated points (deterministic, identical on every rank)."""
        return [tuple(r) for r in gen_points(0, self.cfg.k, self.cfg.blobs, self.cfg.seed).tolist()]

    def iterate(self, cents: list) -> list:
        c = self.ctx.FromEnumerable(cents, dtype=POINT_T)
        return list(step_query(self.points, c))

    def run(self) -> KMeansResult:
        cents = self.initial_centroids()
        times = []
        for _ in range(self.cfg.iterations):
            t0 = time.perf_counter()
            new = self.iterate(cents)
            times.append(time.perf_counter() - t0)
            shift = float(np.abs(np.asarray(new) - np.asarray(cents)).max())
            cents = new
            if shift <= self.cfg.tol:
                break
        return KMeansResult(np.asarray(cents, dtype=np.float32), len(times), times)

    def run_do_while(self) -> np.ndarray:
        """Same iteration through the ``DoWhile`` operator (client loop, one job per iteration)."""
        cfg = self.cfg
        state = {"i": 0}
        c0 = self.ctx.FromEnumerable(self.initial_centroids(), dtype=POINT_T)

        def body(before):
            return step_query(self.points, before)

        def cond(before, after):
            state["i"] += 1
            b, a = np.asarray(list(before)), np.asarray(list(after))
            return state["i"] < cfg.iterations and float(np.abs(a - b).max()) > cfg.tol

        return np.asarray(list(c0.DoWhile(body, cond)), dtype=np.float32)


def reference(cfg: KMeansConfig, partitions: int, iterations: int | None = None) -> np.ndarray:
    """numpy float64 k-means over the same generated points (test oracle for small configs)."""
    from .kmeans_cpu import step_reference
    n = cfg.points_per_partition * partitions
    x = gen_points(0, n, cfg.blobs, cfg.seed)
    c = gen_points(0, cfg.k, cfg.blobs, cfg.seed).astype(np.float64)
    for _ in range(iterations or cfg.iterations):
        s, cnt = step_reference(x, c.astype(np.float32))
        c = np.where(cnt[:, None] > 0, s / np.maximum(cnt, 1)[:, None], c)
        c = c.astype(np.float32).astype(np.float64)
    return c.astype(np.float32)

"""HIP graph capture of launch-bound device loops.

A DryadLINQ job's hot stages are a handful of long kernels over 1e9-row partitions, so launch
overhead does not show there.  It does show in tight iterative loops over small HBM-resident
data (k-means on a few million points, a DoWhile whose body is a few short kernels): each
iteration is a dozen launches + host glue of a few us each against kernels of tens of us.  The
reference has no equivalent (its vertices are processes; an iteration is a whole job,
DryadLinqQueryable.cs:1280-1306 DoWhile); on MI355X the natural tool is a hipGraph: capture the
iteration's launches once on a side stream, then replay the whole chain with one call.

``torch.cuda.CUDAGraph`` is the hipGraph wrapper of PyTorch-ROCm; every launcher in
``dryad_amd.ops`` enqueues on ``torch.cuda.current_stream()`` and never synchronises on the
default path, so the capture sees the kernels themselves.  Capture rules the callers keep:
static input/output buffers (replays read and write the same addresses), no host reads of
device values inside the body, and no allocation that outlives the capture except through
the graph's private memory pool.
"""
from __future__ import annotations

from typing import Callable

import torch


class GraphedLoop:
    """``body()`` repeated ``unroll`` times, captured once and replayed as one hipGraph.

    ``body`` must be capture-safe (see the module docstring).  ``warmup`` eager calls run first
    on the capture stream (lazy kernel attribute setup, workspace allocation) as PyTorch
    requires; they are part of the caller's work, so the caller should count them (or reset its
    state afterwards)."""

    def __init__(self, body: Callable[[], None], unroll: int = 1, warmup: int = 1, device=None):
        if unroll < 1:
            raise ValueError("unroll must be >= 1")
        self.body, self.unroll = body, unroll
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(warmup):
                body()
        torch.cuda.current_stream(self.device).wait_stream(s)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            for _ in range(unroll):
                body()

    def replay(self, times: int = 1) -> None:
        """Enqueue ``times * unroll`` iterations of ``body`` on the current stream."""
        for _ in range(times):
            self.graph.replay()

    def reset(self) -> None:
        self.graph.reset()


class KMeansGraph:
    """Local k-means iterations (assign + partial sums + centroid update) as one hipGraph.

    ``points`` stays resident; ``centroids`` is copied into a static buffer that every replay
    updates in place, ``unroll`` iterations per replay.  Single-partition form of the
    ``KMeansJob`` DoWhile body (models/kmeans.py) for loops whose per-iteration kernels are short
    enough that launches dominate."""

    def __init__(self, points: torch.Tensor, centroids: torch.Tensor, unroll: int = 8):
        from ..ops import kmeans as KM
        self.points = points
        self.c = centroids.detach().to(device=points.device, dtype=torch.float32).contiguous().clone()
        self._c0 = self.c.clone()
        self.ws = KM.KMeansWorkspace(points.shape[0], self.c.shape[0], points.device)

        def body():
            sums, counts, _ = KM.step(self.points, self.c, self.ws)
            self.c.copy_(KM.update(self.c, sums, counts))

        self.loop = GraphedLoop(body, unroll=unroll, warmup=1, device=points.device)
        self.c.copy_(self._c0)          # the warmup iteration ran eagerly: start again from the input
        self.unroll = unroll

    def run(self, iterations: int) -> torch.Tensor:
        """Advance ``iterations`` (a multiple of ``unroll``) iterations; returns the centroids."""
        if iterations % self.unroll:
            raise ValueError(f"iterations ({iterations}) must be a multiple of unroll ({self.unroll})")
        self.loop.replay(iterations // self.unroll)
        return self.c

    def restart(self, centroids: torch.Tensor | None = None) -> None:
        self.c.copy_(self._c0 if centroids is None else centroids.to(self.c.device, torch.float32))

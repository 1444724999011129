"""The per-rank program of a W-rank GPU job, run on ONE GPU ("loopback rank").

An 8-GPU job cannot be rehearsed on a 1-GPU box at full size: RCCL refuses two ranks on one
device, and gloo ranks sharing the GPU would split its HBM.  For plans of the shuffle shape

    stage A (leaf: read -> ... -> hash/range partition)  --cross-->  stage B (... -> output)

this module runs exactly what rank ``r`` of a W-rank job executes, with the SAME device operators
the GPU executor calls (gpu/ops.OPS), and replaces only the all-to-all-v: stage A of rank r is timed
(its read, partial aggregation, partition pass), every other source's stage A is run untimed just
to produce the port slice rank r would receive from it, the slices are laid out in source order
in one receive buffer per column (as parallel/exchange.py lands them), and stage B's program on
that input is timed.  The output (B's last operator before ``output``) stays in HBM for validation.

Reference: the CrossProduct channel between a partitioning stage and its consumer
(GraphBuilder.cs:481-504, DryadLinqQueryGen.cs:2094-2297 for the decomposable GroupBy-Reduce).
"""
from __future__ import annotations

import torch

from ..gpu import ops as G
from ..gpu import stats
from ..gpu.table import DeviceTable, Ported
from ..parallel.comm import World
from .gpu_executor import GpuVertexContext


def shuffle_stages(plan):
    """(stage A, stage B) of a two-stage shuffle plan, or raise ValueError."""
    st = plan.stages
    if len(st) != 2 or st[0].inputs or len(st[1].inputs) != 1 or st[1].inputs[0].kind != "cross" \
            or st[1].inputs[0].src != st[0].id:
        raise ValueError("loopback: the plan is not one leaf stage shuffled into one consumer stage: "
                         + ", ".join(f"{s.id}:{[o['op'] for o in s.ops]}" for s in st))
    return st[0], st[1]


def _copy_table(t: DeviceTable) -> DeviceTable:
    """A table with its own storage (a port slice outlives the producer's buffers)."""
    if t.rows is not None:
        return DeviceTable(t.n, t.shape, rows=t.rows.clone())
    if t.heap is not None or t.strs:
        raise ValueError("loopback: string-bearing shuffles are not simulated")
    cols = {}
    for k, v in t.cols.items():
        cols[k] = v[: t.n].clone()
        stats.inherit(cols[k], v)           # as parallel/exchange.py delivers them: bounds kept
    return DeviceTable(t.n, t.shape, cols)


def _nbytes(t: DeviceTable) -> int:
    if t.rows is not None:
        return t.rows[: t.n].numel()
    return sum(v[: t.n].numel() * v.element_size() for v in t.cols.values())


class LoopbackRank:
    """Rank ``rank`` of a ``W``-rank run of ``plan`` (compiled with PartitionCount = W) on
    ``device``.  ``step()`` returns the phase timings (ms); ``out`` holds stage B's result."""

    def __init__(self, plan, W: int, rank: int, device=None):
        self.plan, self.W, self.rank = plan, W, rank
        self.dev = torch.device(device or "cuda")
        self.A, self.B = shuffle_stages(plan)
        if self.A.partitions != W or self.B.partitions != W:
            raise ValueError("loopback: compile the plan with PartitionCount = W")
        self.world = World(rank=rank, size=W, local_rank=0, device=self.dev, backend=None)
        self.out = None
        self.phases = {}
        self.bytes = {}

    def _ctx(self, s, p):
        return GpuVertexContext(p, s.partitions, 0, 0, s, self.dev, self.world, None)

    def _run(self, s, p, data, ops):
        v = self._ctx(s, p)
        for op in ops:
            fn = G.OPS.get(op["op"])
            if fn is None:
                raise ValueError(f"loopback: no device operator for {op['op']}")
            data = fn(op, [data] if data is not None else [], v)
        return data

    def step(self) -> dict:
        W, me, A, B = self.W, self.rank, self.A, self.B
        # the previous step's output is not kept through this one (a real rank hands it on): held,
        # it crowded stage B's allocations into fresh segments (a 1.8 s stage B, one step in four)
        self.out = None
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        torch.cuda.reset_peak_memory_stats(self.dev)
        base = torch.cuda.memory_allocated(self.dev)
        ev[0].record()
        mine = self._run(A, me, None, A.ops)                 # read -> ... -> partition: this rank's work
        ev[1].record()
        peak_a = torch.cuda.max_memory_allocated(self.dev) - base
        if not isinstance(mine, Ported):
            raise ValueError("loopback: stage A does not end in a partitioning operator")
        sent = sum(_nbytes(mine.port(p)) for p in range(mine.nports) if p % W != me)
        # the exchange, simulated (untimed): every source's piece for this rank, in source order
        pieces = []
        for s in range(W):
            src = mine if s == me else self._run(A, s, None, A.ops)
            pieces.append(_copy_table(src.port(me)))
            del src
        recv = DeviceTable.concat(pieces)
        if recv.rows is None:
            cols = {}
            for k, v in recv.cols.items():
                cols[k] = v.contiguous()
                stats.inherit(cols[k], v)
            recv = DeviceTable(recv.n, recv.shape, cols)
        del pieces, mine
        recv_bytes = _nbytes(recv)
        ops = [o for o in B.ops if o["op"] != "output"]
        torch.cuda.synchronize(self.dev)
        torch.cuda.reset_peak_memory_stats(self.dev)
        base_b = torch.cuda.memory_allocated(self.dev)
        ev[2].record()
        self.out = self._run(B, me, recv, ops)
        ev[3].record()
        torch.cuda.synchronize(self.dev)
        peak_b = torch.cuda.max_memory_allocated(self.dev) - base_b + recv_bytes
        self.phases = {"stage_a_ms": ev[0].elapsed_time(ev[1]), "stage_b_ms": ev[2].elapsed_time(ev[3])}
        # HBM working set of each timed stage (caching-allocator peaks above what was live before
        # it; stage B counts the received table it consumes)
        self.bytes = {"sent_bytes": sent, "received_bytes": recv_bytes, "received_rows": recv.n,
                      "hbm_stage_a_GB": round(peak_a / 1e9, 2), "hbm_stage_b_GB": round(peak_b / 1e9, 2)}
        return self.phases

    @property
    def ms(self) -> float:
        return sum(self.phases.values())

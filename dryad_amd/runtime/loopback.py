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


def _arena_table(arena, tabs: list):
    """The round's received pieces laid into the next region of the receive arena (what the
    exchange's all-to-all-v writes there in a real run), or None (strings, rows, no room)."""
    if not tabs or any(t.rows is not None or t.heap is not None or t.strs for t in tabs):
        return None
    t0 = tabs[0]
    n = sum(t.n for t in tabs)
    dts, widths = {}, {}
    for k, v in t0.cols.items():
        dt = v.dtype
        for t in tabs[1:]:
            dt = torch.promote_types(dt, t.cols[k].dtype)
        dts[k] = (dt, tuple(v.shape[1:]))
        w = torch.empty((0,) + tuple(v.shape[1:]), dtype=dt).element_size()
        for d in v.shape[1:]:
            w *= d
        widths[k] = w
    slots = arena.take(widths, n)
    if slots is None:
        return None
    cols = {}
    for k, (dt, tail) in dts.items():
        dst = slots[k].view(dt).view((n,) + tail)
        a = 0
        for t in tabs:
            dst[a: a + t.n].copy_(t.cols[k][: t.n])
            a += t.n
        stats.union(dst, [t.cols[k] for t in tabs])
        cols[k] = dst
    return DeviceTable(n, t0.shape, cols)


def bulk_model(phases: dict, nbytes: dict, link_GBps: float) -> dict:
    """MODELLED step of the bulk plan (stage A, one exchange, stage B) on a link of ``link_GBps``
    per GPU: the exchange takes max(bytes out, bytes in) / link between the two stages."""
    wire = max(nbytes["sent_bytes"], nbytes["received_bytes"]) / (link_GBps * 1e6)
    return dict(link_GBps=link_GBps, modelled=True, wire_ms=round(wire, 2),
                step_ms=round(phases["stage_a_ms"] + wire + phases["stage_b_ms"], 2))


class LoopbackStreamShuffle:
    """Rank ``rank`` of a W-rank streamed shuffle (runtime/stream_shuffle.py) on one GPU: per round,
    this rank's chunk through stage A's program (read chunk, record-wise ops, partial aggregation,
    hash partition) and the fold of the round's received pieces into stage B's running state are
    timed; the pieces the other W - 1 sources would send it in that round are produced untimed by
    running their chunk of the round.  ``model(link)`` replays the measured per-round times in the
    streamed shuffle's queue order with each round's exchange taking max(bytes out, bytes in) /
    link (MODELLED: no link is measured here)."""

    def __init__(self, plan, W: int, rank: int, ctx, device=None):
        from . import stream_shuffle as SSH
        self.plan, self.W, self.rank, self.ctx = plan, W, rank, ctx
        self.dev = torch.device(device or "cuda")
        self.A, self.B = shuffle_stages(plan)
        if self.A.partitions != W:
            raise ValueError("loopback: compile the plan with PartitionCount = W")
        d = SSH.find(plan).get(self.B.id)
        if d is None:
            raise ValueError("loopback: the plan is not a streamed-shuffle pair")
        self.world = World(rank=rank, size=W, local_rank=0, device=self.dev, backend=None)
        self.out = None
        self.rounds = []

    def _splan(self):
        from . import stream_agg as SA
        from . import streaming as ST
        props = self.ctx._props

        class _R:                      # the minimal runner surface streaming._source / budget read
            pass
        r = _R()
        r.ctx, r.dev = self.ctx, self.dev
        src = ST._source(r, self.A)
        budget = int(props.get("HbmBudgetBytes") or torch.cuda.mem_get_info(self.dev)[0] * 0.8)
        chunk = max(1 << 20, min(int(props.get("StreamChunkBytes") or ST.DEFAULT_CHUNK_BYTES), budget // 8))
        big = ST._partition_bytes(src[0], src[1], self.rank)
        return dict(kind=src[0], info=src[1], chunk=chunk, budget=budget, source_bytes=big,
                    pre=self.A.ops[1:-2], agg=self.A.ops[-2], rest=self.A.ops[-1:]), SA

    def _a_round(self, s, t):
        v = GpuVertexContext(s, self.A.partitions, 0, 0, self.A, self.dev, self.world, None)
        data = t
        for op in self.A.ops[1:]:
            data = G.OPS[op["op"]](op, [data], v)
        return data                  # Ported

    def step(self) -> dict:
        from . import streaming as ST
        W, me = self.W, self.rank
        self.out = None
        splan, SA = self._splan()
        vb = GpuVertexContext(me, self.B.partitions, 0, 0, self.B, self.dev, self.world, None)

        class _Runner:               # what StreamAggregator and finish() use of the executor
            pass
        run = _Runner()
        run.ctx, run.dev, run.stream_stats = self.ctx, self.dev, {}
        run._run_op = lambda op, ins, v, s: G.OPS[op["op"]](op, ins, v)
        bplan = dict(agg=self.B.ops[0], pre=[], rest=[], budget=splan["budget"], source_bytes=splan["source_bytes"],
                     hold_bytes=splan["budget"] // 4,
                     chunk=splan["chunk"])
        agg = SA.StreamAggregator(run, self.B, vb, bplan)
        from ..parallel import exchange as EXC
        arena = EXC.RecvArena(bplan["hold_bytes"], self.dev)      # as stream_shuffle.run receives
        gens = [ST._chunks(splan, s, self.dev, None) for s in range(W)]
        self.rounds = []
        t_all = torch.cuda.Event(enable_timing=True)
        t_all.record()
        while True:
            mine = next(gens[me], None)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            ev[0].record()
            ported = self._a_round(me, mine) if mine is not None else None
            ev[1].record()
            pieces = []
            sent = 0
            if ported is not None:
                sent = sum(_nbytes(ported.port(p)) for p in range(ported.nports) if p != me)
                pieces.append((me, _copy_table(ported.port(me))))
            others = False
            for s in range(W):               # the round's pieces from the other sources (untimed)
                if s == me:
                    continue
                t = next(gens[s], None)
                if t is None:
                    continue
                others = True
                pieces.append((s, _copy_table(self._a_round(s, t).port(me))))
            if mine is None and not others:
                break
            pieces.sort(key=lambda x: x[0])
            tabs = [p for _, p in pieces if p.n]
            recv = _arena_table(arena, tabs)
            if recv is None:
                recv = DeviceTable.concat(tabs) if len(tabs) > 1 else (tabs[0] if tabs else None)
            rb = _nbytes(recv) - (_nbytes(pieces[0][1]) if pieces and pieces[0][0] == me else 0) if recv else 0
            torch.cuda.synchronize(self.dev)
            ev[2].record()
            if recv is not None:
                agg.add_partial(recv)
            ev[3].record()
            torch.cuda.synchronize(self.dev)
            self.rounds.append(dict(a_ms=ev[0].elapsed_time(ev[1]), fold_ms=ev[2].elapsed_time(ev[3]),
                                    sent_bytes=sent, recv_bytes=rb))
            del pieces, recv, ported
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        res = list(agg.bucket_results(True))
        self.out = DeviceTable.concat(res) if len(res) > 1 else (res[0] if res else None)
        e1.record()
        torch.cuda.synchronize(self.dev)
        self.finish_ms = e0.elapsed_time(e1)
        self.stats = dict(agg.stats, buckets=agg.K, spilled_buckets=len(agg.spilled))
        self.phases = {"rounds": len(self.rounds), "stage_a_ms": sum(r["a_ms"] for r in self.rounds),
                       "fold_ms": sum(r["fold_ms"] for r in self.rounds), "finish_ms": self.finish_ms}
        return self.phases

    @property
    def ms(self) -> float:
        return self.phases["stage_a_ms"] + self.phases["fold_ms"] + self.phases["finish_ms"]

    def model(self, link_GBps: float) -> dict:
        """Queue order of stream_shuffle.run: A(r), exchange(r) queued, fold(r - 1) (waits for
        round r - 1), ..., fold(R - 1), finish; one compute stream, one link."""
        comp = comm = 0.0
        end = []
        for r, rd in enumerate(self.rounds):
            comp += rd["a_ms"]
            start = max(comp, comm)
            end.append(start + max(rd["sent_bytes"], rd["recv_bytes"]) / (link_GBps * 1e6))
            comm = end[-1]
            if r >= 1:
                comp = max(comp, end[r - 1]) + self.rounds[r - 1]["fold_ms"]
        if self.rounds:
            comp = max(comp, end[-1]) + self.rounds[-1]["fold_ms"]
        comp += self.finish_ms
        wire = sum(max(r["sent_bytes"], r["recv_bytes"]) for r in self.rounds) / (link_GBps * 1e6)
        return dict(link_GBps=link_GBps, modelled=True, wire_ms=round(wire, 2), step_ms=round(comp, 2))

"""Streamed, out-of-core GroupBy / Distinct: a partition larger than the HBM budget aggregated in
bounded chunks.

The reference never holds a GroupBy partition: its partial accumulation consumes the input
stream into a hash table (ParallelHashGroupByPartialAccumulate, LinqToDryad/DryadLinqVertex.cs:5718)
and its sort spills to FileEnumerable (:9584-9615, 10733).  Here the stage's source is read in
chunks (runtime/streaming._chunks: generator sub-ranges, stored rows, fixed-width part ranges),
and every chunk goes through the stage's record-wise operators and the device partial aggregation
(gpu/ops.op_group_partial: LDS hash tables, dense or radix aggregation) or Distinct.  The chunk's
partial rows are split into K hash buckets (one stable column scatter) and appended to their
bucket; a bucket whose pending pieces reach its running state's size is folded with it
(gpu/ops.combine_partials, the RecursiveAccumulate), so a bucket holds about one row per distinct
key of its hash range.  When the buckets' states outgrow the HBM budget the largest go to pinned
host memory, and their later pieces follow them there.  At the end each bucket is folded once
more and reduced (FinalReduce) on its own, in HBM bounded by one bucket, and the results are
concatenated (or, for a Distinct / GroupBy feeding a partitioning op, the folded partials are).

Plans: a leaf stage ``read -> (Select | Where)* -> group_by(decomposable) | distinct -> ...`` (a
partition already keyed, e.g. one rank) or ``read -> ... -> group_partial -> hash_partition`` (the
partial side of a multi-rank GroupBy: the folded partials then go through the exchange).  Chosen
when the source partition exceeds ``HbmBudgetBytes`` (context property; default 80% of free HBM)
or ``StreamAggregate=True``.
"""
from __future__ import annotations

import time

import torch

from ..gpu import ops as G
from ..gpu.table import DeviceTable, Shape
from ..ops import relational as R
from ..utils.log import get_logger
from . import streaming as ST

log = get_logger("stream_agg")

PRE_OPS = {"select", "where", "identity"}
AGG_OPS = {"group_by", "group_partial", "distinct"}


def plan(runner, s):
    """The streamed-aggregation plan of stage s, or None."""
    if not runner.gpu_ok or s.inputs or len(s.ops) < 2 or s.id in runner.skipped or s.id in runner.gang_stages:
        return None
    src = ST._source(runner, s)
    if src is None:
        return None
    k = next((i for i, o in enumerate(s.ops[1:], 1) if o["op"] not in PRE_OPS), None)
    if k is None or s.ops[k]["op"] not in AGG_OPS:
        return None
    agg = s.ops[k]
    if agg["op"] in ("group_by", "group_partial") and (agg.get("decomp") is None or agg.get("elem") is not None
                                                       or agg.get("comparer") is not None):
        return None
    if agg["op"] == "distinct" and agg.get("comparer") is not None:
        return None
    rest = s.ops[k + 1:]
    if agg["op"] == "group_partial" and [o["op"] for o in rest] not in (["hash_partition"], []):
        return None
    props = runner.ctx._props
    force = props.get("StreamAggregate")
    if force is False:
        return None
    budget = _budget(runner)
    big = max((ST._partition_bytes(src[0], src[1], p) for p in range(s.partitions)), default=0)
    if not force and big <= budget:
        return None
    chunk = int(props.get("StreamChunkBytes") or ST.DEFAULT_CHUNK_BYTES)
    chunk = max(1 << 20, min(chunk, budget // 8))
    return dict(kind=src[0], info=src[1], chunk=chunk, pre=s.ops[1:k], agg=agg, rest=rest, budget=budget,
                source_bytes=big)


def _budget(runner) -> int:
    b = runner.ctx._props.get("HbmBudgetBytes")
    if b:
        return int(b)
    free, _ = torch.cuda.mem_get_info(runner.dev)
    return int(free * 0.8)


def _nbytes(t) -> int:
    if t is None:
        return 0
    if isinstance(t, HostPiece):
        return t.nbytes
    if t.rows is not None:
        return t.rows[: t.n].numel()
    return sum(v[: t.n].numel() * v.element_size() for v in t.cols.values())


class HostPiece:
    """A table's columns in pinned host memory (a spilled bucket state or piece)."""

    def __init__(self, t: DeviceTable):
        self.n, self.shape, self.strs = t.n, t.shape, t.strs
        self.rows = None
        self.cols = {}
        if t.rows is not None:
            self.rows = torch.empty(t.rows[: t.n].shape, dtype=t.rows.dtype, pin_memory=True)
            self.rows.copy_(t.rows[: t.n], non_blocking=True)
        for k, v in t.cols.items():
            h = torch.empty(v[: t.n].shape, dtype=v.dtype, pin_memory=True)
            h.copy_(v[: t.n], non_blocking=True)
            self.cols[k] = h
        self.nbytes = _nbytes(t)

    def to_device(self, dev) -> DeviceTable:
        if self.rows is not None:
            return DeviceTable(self.n, self.shape, rows=self.rows.to(dev, non_blocking=True))
        return DeviceTable(self.n, self.shape, {k: v.to(dev, non_blocking=True) for k, v in self.cols.items()})


def _key_fields(t: DeviceTable, agg_kind: str):
    """Hash key fields of a partial table (its key columns) or of whole records (Distinct)."""
    if agg_kind != "distinct":
        nk = t.shape.pytype.nkeys
        return [R.HashKey.column(t.cols[f"k{i}"]) for i in range(nk)], nk > 1
    if t.rows is not None:
        return [R.HashKey.bytes_field(t.rows, 0, t.rows.shape[1])], False
    if t.heap is not None or t.strs:
        raise G.NotTraceable("streamed Distinct of records with strings")
    cols = [t.cols[f] for f in t.shape.fields]
    return [R.HashKey.column(c) for c in cols], len(cols) > 1


def _buckets(t: DeviceTable, K: int, agg_kind: str) -> list:
    """t split into K hash buckets (one stable column scatter) -> list of K slices."""
    if t.n == 0:
        return [None] * K
    keys, tup = _key_fields(t, agg_kind)
    _, hs = R.stable_hash_dest(keys, t.n, 0, tup, t.device, want_hash=True)
    # bucket from bits of the mixed hash the rank partitioner (h mod W) does not use
    b = ((hs * -7046029254386353131) >> 40) & 0xFFFFFF
    ports = (b % K).to(torch.uint8)
    from ..ops import channel as CH
    cols = [t.rows] if t.rows is not None else list(t.cols.values())
    outs, cnt = CH.scatter_columns(ports, t.n, cols)
    off = [0]
    for c in cnt[:K].tolist():
        off.append(off[-1] + int(c))
    nt = DeviceTable(t.n, t.shape, rows=outs[0]) if t.rows is not None else \
        DeviceTable(t.n, t.shape, dict(zip(t.cols.keys(), outs)))
    return [nt.slice(off[k], off[k + 1]) if off[k + 1] > off[k] else None for k in range(K)]


class StreamAggregator:
    """Bounded-HBM GroupBy / Distinct over a stream of chunks (see the module docstring)."""

    def __init__(self, runner, s, vctx, splan):
        self.runner, self.s, self.v, self.p = runner, s, vctx, splan
        self.agg = splan["agg"]
        self.kind = "distinct" if self.agg["op"] == "distinct" else "group"
        self.d = self.agg.get("decomp")
        self.budget = splan["budget"]
        self.K = None
        self.state: list = []          # per bucket: DeviceTable | HostPiece | None
        self.pending: list = []        # per bucket: [DeviceTable | HostPiece]
        self.spilled: set = set()
        self.stats = dict(chunks=0, records_in=0, combines=0, spilled_bytes=0, spill_events=0)

    # ------------------------------------------------------------------ per chunk
    def _partial(self, t: DeviceTable) -> DeviceTable:
        if self.kind == "distinct":
            return G.op_distinct(self.agg, [t], self.v)
        op = dict(self.agg, op="group_partial")
        return G.op_group_partial(op, [t], self.v)

    def _fold(self, pieces: list) -> DeviceTable:
        dev = self.v.device
        tabs = [x.to_device(dev) if isinstance(x, HostPiece) else x for x in pieces if x is not None]
        tabs = [x for x in tabs if x.n]
        if not tabs:
            return None
        t = DeviceTable.concat(tabs) if len(tabs) > 1 else tabs[0]
        if t.rows is None:
            t = DeviceTable(t.n, t.shape, {k: v[: t.n].contiguous() for k, v in t.cols.items()})
        self.stats["combines"] += 1
        if self.kind == "distinct":
            return G.op_distinct(self.agg, [t], self.v)
        return G.combine_partials(t, self.d)

    def _choose_buckets(self, part: DeviceTable, rows_in: int):
        """K from the source size: every bucket's folded state must fit a quarter of the budget
        even if partial aggregation reduced nothing (2^k, 16..256)."""
        per_row = _nbytes(part) / max(part.n, 1)
        total_rows = max(rows_in, 1) * self.p["source_bytes"] / max(self.p["chunk_bytes_first"], 1)
        want = per_row * total_rows / max(self.budget // 4, 1)
        K = 16
        while K < 256 and K < want:
            K *= 2
        self.K = K
        self.state = [None] * K
        self.pending = [[] for _ in range(K)]

    def _resident(self) -> int:
        tot = 0
        for k in range(self.K):
            if k not in self.spilled:
                tot += _nbytes(self.state[k]) + sum(_nbytes(x) for x in self.pending[k])
        return tot

    def _spill(self):
        """Largest HBM-resident buckets -> pinned host memory until the resident set is back
        under half the budget."""
        order = sorted((k for k in range(self.K) if k not in self.spilled),
                       key=lambda k: -(_nbytes(self.state[k]) + sum(_nbytes(x) for x in self.pending[k])))
        for k in order:
            if self._resident() <= self.budget // 2:
                break
            moved = 0
            if self.state[k] is not None and not isinstance(self.state[k], HostPiece):
                self.state[k] = HostPiece(self.state[k])
                moved += self.state[k].nbytes
            self.pending[k] = [HostPiece(x) if not isinstance(x, HostPiece) else x for x in self.pending[k]]
            moved += sum(x.nbytes for x in self.pending[k])
            self.spilled.add(k)
            self.stats["spilled_bytes"] += moved
            self.stats["spill_events"] += 1
        torch.cuda.synchronize(self.v.device)

    def add_chunk(self, t: DeviceTable):
        self.stats["chunks"] += 1
        self.stats["records_in"] += t.n
        data = t
        for op in self.p["pre"]:
            data = self.runner._run_op(op, [data], self.v, self.s)
        if data is None or data.n == 0:
            return
        part = self._partial(data)
        if self.K is None:
            self.p["chunk_bytes_first"] = _nbytes(t)
            self._choose_buckets(part, t.n)
        for k, piece in enumerate(_buckets(part, self.K, self.kind)):
            if piece is None:
                continue
            if k in self.spilled:
                self.pending[k].append(HostPiece(piece))
                continue
            self.pending[k].append(piece)
            if sum(_nbytes(x) for x in self.pending[k]) >= max(_nbytes(self.state[k]), self.budget // (8 * self.K)):
                self.state[k] = self._fold([self.state[k]] + self.pending[k])
                self.pending[k] = []
        del part
        if self._resident() > int(self.budget * 0.7):
            self._spill()

    # ------------------------------------------------------------------ end of stream
    def bucket_results(self, final: bool):
        """Yield each bucket's folded state (``final``: reduced to the GroupBy's result)."""
        for k in range(self.K or 0):
            t = self._fold([self.state[k]] + self.pending[k])
            self.state[k], self.pending[k] = None, []
            if t is None or t.n == 0:
                continue
            if final and self.kind == "group":
                t = G.final_reduce(t, self.d)
            yield t


def run(runner, s, p, version, vctx, splan):
    """Run stage s's partition p as a streamed aggregation -> the stage's output value."""
    t0 = time.perf_counter()
    agg = StreamAggregator(runner, s, vctx, splan)
    for chunk in ST._chunks(splan, p, vctx.device, vctx):
        agg.add_chunk(chunk)
    t1 = time.perf_counter()
    final = splan["agg"]["op"] != "group_partial"
    pieces = list(agg.bucket_results(final))
    if pieces:
        out = DeviceTable.concat(pieces)
    else:
        out = _empty_result(runner, s, vctx, splan)
    for op in splan["rest"]:
        out = runner._run_op(op, [out], vctx, s)
    runner.stream_stats[(s.id, p)] = dict(agg.stats, buckets=agg.K, spilled_buckets=len(agg.spilled),
                                           stream_s=round(t1 - t0, 3),
                                           finish_s=round(time.perf_counter() - t1, 3),
                                           budget_bytes=agg.budget, kind="streamed aggregation")
    return out


def _empty_result(runner, s, vctx, splan):
    """An empty input partition: the operators' own empty result (host path records nothing)."""
    return []

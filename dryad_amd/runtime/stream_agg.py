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
    """A table's columns in pinned host memory (a spilled bucket state or piece), in leased
    exact-size page-locked buffers (ops/_lib.pinned_lease: reused by later spills and by the
    streamed result, not rounded up to a power of two like torch's pinned allocator).  Every copy
    in and out is ordered on the current stream, so ``release()`` may hand the buffers on as soon
    as the copy out is queued."""

    def __init__(self, t: DeviceTable):
        from ..ops._lib import pinned_lease
        self.n, self.shape, self.strs = t.n, t.shape, t.strs
        self.rows = None
        self.cols = {}
        self.leases = []

        def out(v):
            ls = pinned_lease(tuple(v.shape), v.dtype)
            ls.tensor.copy_(v, non_blocking=True)
            self.leases.append(ls)
            return ls.tensor
        if t.rows is not None:
            self.rows = out(t.rows[: t.n])
        for k, v in t.cols.items():
            self.cols[k] = out(v[: t.n])
        self.nbytes = _nbytes(t)

    def to_device(self, dev) -> DeviceTable:
        if self.rows is not None:
            return DeviceTable(self.n, self.shape, rows=self.rows.to(dev, non_blocking=True))
        return DeviceTable(self.n, self.shape, {k: v.to(dev, non_blocking=True) for k, v in self.cols.items()})

    def release(self):
        for ls in self.leases:
            ls.release()
        self.leases, self.rows, self.cols = [], None, {}


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


class DenseState:
    """Running GroupBy state of ONE integer key addressed directly by key - lo: one slot per key
    of the keys' range and accumulator (8-byte accumulators side by side per key: one HBM sector
    per folded row; sums and counts added, min / max reduced into their slots), plus an occupancy
    byte unless a count accumulator tells occupancy.  Used while the range times
    the slot bytes fits DENSE_FRACTION of the budget (e.g. 2^30 keys x 33 bytes = 35 GB of a 60 GB
    budget): a chunk's partial rows then fold into the state in place (ops/densegroup
    .dense_state_update: one pass of atomics per row), with no hash buckets,
    pending pieces, combines or spills.  The range grows (coarsely aligned) as chunks reach past it;
    when it no longer fits, the state becomes one partial piece of the hash-bucket path."""

    DENSE_FRACTION = 0.75

    def __init__(self, d, budget: int):
        self.d, self.cap = d, int(budget * self.DENSE_FRACTION)
        self.lo = self.hi = None
        self.specs = None            # [(state name, op, source column name or None, dtype)]
        self.state = {}              # [R, S] int64 matrix (aos) or {name: [R] array}
        self.seen = None             # occupancy bytes, unless a count accumulator tells it
        self.aos = False
        self.count_name = None
        self.meta = None
        self.kdtype = None
        self.outdt: dict = {}

    @staticmethod
    def eligible(part: DeviceTable) -> bool:
        m = part.shape.pytype
        k = part.cols.get("k0") if part.rows is None else None
        return (part.shape.kind == "partial" and not part.strs and getattr(m, "nkeys", 0) == 1 and k is not None
                and k.dtype in (torch.int8, torch.int16, torch.int32, torch.int64))

    def _plan(self, part: DeviceTable):
        """Accumulator layout, fixed by the first chunk.  Count accumulators are recorded as
        "count" here; whether a chunk's count column is implicit (a raw partial: int8 ones) or a
        folded count to be summed is decided per chunk (``_chunk_specs``), because the partial step
        may emit raw rows for one chunk and folded rows for the next."""
        specs = []
        for j, a in enumerate(self.d.aggs):
            col = part.cols.get(f"a{j}")
            if a.kind == "count":
                specs.append((f"a{j}", "count", None, torch.int64))
                self.outdt[f"a{j}"] = torch.int64
            elif a.kind == "sum":
                dt = torch.float64 if col.dtype.is_floating_point else torch.int64
                specs.append((f"a{j}", "sum", f"a{j}", dt))
                self.outdt[f"a{j}"] = dt
            elif a.kind in ("min", "max"):
                specs.append((f"a{j}", a.kind, f"a{j}", col.dtype))
                self.outdt[f"a{j}"] = col.dtype
            elif a.kind == "avg":
                c = part.cols.get(f"c{j}")
                specs.append((f"a{j}", "sum", f"a{j}", torch.float64))
                specs.append((f"c{j}", "count", None, torch.int64))
                self.outdt[f"a{j}"], self.outdt[f"c{j}"] = torch.float64, torch.int64
            else:
                return None              # any / all / user aggregates: the bucket path
        return specs

    def _chunk_specs(self, part: DeviceTable):
        """The specs for one chunk: a count accumulator sums the chunk's count column when it is a
        folded count (wider than int8), and adds one per row when the column is absent or holds
        the raw partial's int8 ones."""
        out = []
        for name, op, src, dt in self.specs:
            if op == "count":
                col = part.cols.get(name)
                if col is not None and col.dtype != torch.int8:
                    op, src = "sum", name
            out.append((name, op, src, dt))
        return out

    def _layout(self):
        """8-byte accumulators only: one [R, S] matrix, a key's S slots side by side (its folds touch
        one HBM sector instead of S); a count accumulator doubles as the occupancy flag."""
        self.aos = all(dt in (torch.int64, torch.float64) for _, _, _, dt in self.specs)
        cnt = {f"a{j}" for j, a in enumerate(self.d.aggs) if a.kind == "count"} | \
            {f"c{j}" for j, a in enumerate(self.d.aggs) if a.kind == "avg"}
        self.count_name = next((name for name, _, _, _ in self.specs if name in cnt), None)

    def _slot_bytes(self) -> int:
        return (0 if self.count_name else 1) + sum(torch.empty(0, dtype=dt).element_size() for _, _, _, dt in self.specs)

    def _col(self, st, name: str):
        """The state column of accumulator ``name`` (a strided view of the matrix, or its array)."""
        if not self.aos:
            return st[name]
        s = self.slot[name]
        dt = self.dtypes[name]
        return (st if dt == torch.int64 else st.view(dt))[:, s]

    def _alloc(self, lo: int, hi: int, dev):
        R = hi - lo + 1
        if self.aos:
            st = torch.empty((R, len(self.specs)), dtype=torch.int64, device=dev)
        else:
            st = {name: torch.empty(R, dtype=dt, device=dev) for name, _, _, dt in self.specs}
        for name, op, _, dt in self.specs:
            if op == "min":
                fill = torch.iinfo(dt).max if not dt.is_floating_point else float("inf")
            elif op == "max":
                fill = torch.iinfo(dt).min if not dt.is_floating_point else float("-inf")
            else:
                fill = 0
            self._col(st, name).fill_(fill)
        seen = None if self.count_name else torch.zeros(R, dtype=torch.int8, device=dev)
        if self.lo is not None:          # the old range moves into the grown one
            a, b = self.lo - lo, self.hi - lo + 1
            if self.aos:
                st[a:b].copy_(self.state)
            else:
                for name in st:
                    st[name][a:b].copy_(self.state[name])
            if seen is not None:
                seen[a:b].copy_(self.seen)
        self.state, self.seen, self.lo, self.hi = st, seen, lo, hi

    def add(self, part: DeviceTable) -> bool:
        """Fold a chunk's partial rows in; False when its keys' range would not fit (the caller
        moves to the hash buckets)."""
        n = part.n
        if n == 0:
            return True
        if self.specs is None:
            self.specs = self._plan(part)
            self.meta = part.shape.pytype
            self.kdtype = part.cols["k0"].dtype
            if self.specs is None:
                return False
            self.slot = {name: i for i, (name, _, _, _) in enumerate(self.specs)}
            self.dtypes = {name: dt for name, _, _, dt in self.specs}
            self._layout()
        k = part.cols["k0"][:n]
        mn, mx = (int(x) for x in torch.aminmax(k))
        lo, hi = (mn, mx) if self.lo is None else (min(mn, self.lo), max(mx, self.hi))
        if self.lo is None or lo < self.lo or hi > self.hi:
            span = hi - lo + 1
            g = 1 << max(0, span.bit_length() - 4)        # coarse alignment: few regrowths
            alo, ahi = (lo // g) * g, -(-(hi + 1) // g) * g - 1
            if (ahi - alo + 1) * self._slot_bytes() <= self.cap:
                lo, hi = alo, ahi
            if (hi - lo + 1) * self._slot_bytes() > self.cap:
                return False
            self._alloc(lo, hi, k.device)
        from ..ops import densegroup as DG
        specs = self._chunk_specs(part)
        fused = [(self._col(self.state, name), op, part.cols[src][:n] if src is not None else None)
                 for name, op, src, _ in specs]
        stride = len(self.specs) if self.aos else 1
        if DG.dense_state_ok(fused, k, stride):
            # one pass, every accumulator
            DG.dense_state_update(k, self.lo, self.seen, fused, rng=self.hi - self.lo + 1, stride=stride)
            return True
        idx = (k - self.lo).to(torch.int64)
        if self.seen is not None:
            self.seen.index_fill_(0, idx, 1)
        for name, op, src, dt in specs:
            st = self._col(self.state, name)
            if op == "count":
                st.index_add_(0, idx, torch.ones(1, dtype=dt, device=st.device).expand(n))
                continue
            v = part.cols[src][:n]
            v = v if v.dtype == dt else v.to(dt)
            if op == "sum":
                st.index_add_(0, idx, v)
            else:
                st.scatter_reduce_(0, idx, v, reduce="amin" if op == "min" else "amax", include_self=True)
        return True

    def nbytes(self) -> int:
        return 0 if self.lo is None else (self.hi - self.lo + 1) * self._slot_bytes()

    def to_partial(self) -> DeviceTable | None:
        """The occupied slots as a partial table in the folded (standard) layout."""
        if self.lo is None:
            return None
        occupied = self.seen if self.seen is not None else self._col(self.state, self.count_name)
        occ = torch.nonzero(occupied).squeeze(1)
        out = {"k0": (occ + self.lo).to(self.kdtype)}
        for name, _, _, _ in self.specs:
            out[name] = self._col(self.state, name).index_select(0, occ)
        for j, a in enumerate(self.d.aggs):      # min / max keep their dtype (as combine_partials)
            if a.kind in ("min", "max") and out[f"a{j}"].dtype != self.outdt[f"a{j}"]:
                out[f"a{j}"] = out[f"a{j}"].to(self.outdt[f"a{j}"])
        self.state, self.seen = {}, None
        from ..gpu.table import PartialMeta
        m = self.meta
        meta = PartialMeta(m.nkeys, m.kinds, m.key_form)
        return DeviceTable.from_columns(out, Shape("partial", list(out), meta))


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
        # GroupBy of one integer key: the directly addressed running state while it fits
        use = runner.ctx._props.get("StreamDenseState", True) and self.kind == "group"
        self.dense = DenseState(self.d, self.budget) if use else None
        # received partials of a streamed shuffle (add_partial) held in HBM up to ``hold_bytes`` and
        # combined once per batch by the partition + LDS aggregation of a final GroupBy (the bulk
        # path's kernels) instead of folded round by round into the running state with per-row
        # atomics: with one batch the whole fold is one final reduce after the last round
        self.hold_budget = int(splan.get("hold_bytes") or 0) if self.kind == "group" else 0
        self.held, self.held_bytes, self.direct = [], 0, None

    # ------------------------------------------------------------------ per chunk
    def _partial(self, t: DeviceTable) -> DeviceTable:
        if self.kind == "distinct":
            return G.op_distinct(self.agg, [t], self.v)
        op = dict(self.agg, op="group_partial")
        if self.dense is not None:
            op["raw_ok"] = True      # mostly distinct keys: the dense state folds the raw rows itself
        return G.op_group_partial(op, [t], self.v)

    def _fold(self, pieces: list) -> DeviceTable:
        dev = self.v.device
        tabs = [x.to_device(dev) if isinstance(x, HostPiece) else x for x in pieces if x is not None]
        for x in pieces:                 # (their copies to HBM are queued: the buffers go back to the pool)
            if isinstance(x, HostPiece):
                x.release()
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
        if "chunk_bytes_first" not in self.p:
            self.p["chunk_bytes_first"] = _nbytes(t)
        data = t
        for op in self.p["pre"]:
            data = self.runner._run_op(op, [data], self.v, self.s)
        if data is None or data.n == 0:
            return
        self._fold_in(self._partial(data), t.n)

    def add_partial(self, part: DeviceTable):
        """Fold in a table of partial rows another stage produced (the received rounds of a
        streamed shuffle, runtime/stream_shuffle.py): GroupBy partials go straight into the running
        state; records of a Distinct are deduplicated first."""
        if part is None or part.n == 0:
            return
        self.stats["chunks"] += 1
        self.stats["records_in"] += part.n
        if "chunk_bytes_first" not in self.p:
            self.p["chunk_bytes_first"] = _nbytes(part)
        if self.kind == "distinct":
            part = G.op_distinct(self.agg, [part], self.v)
        if self.hold_budget:
            nb = _nbytes(part)
            if self.held_bytes + nb > self.hold_budget:
                self._flush_held()
            if nb <= self.hold_budget:
                self.held.append(part)
                self.held_bytes += nb
                return
        self._fold_in(part, part.n)

    def _state_only_direct(self) -> bool:
        return self.K is None and (self.dense is None or self.dense.nbytes() == 0)

    def _state_empty(self) -> bool:
        return self.K is None and (self.dense is None or self.dense.nbytes() == 0) and self.direct is None

    def _flush_held(self):
        """The held partials combined into one partial row per key: kept as is while nothing else
        is held (the common case: every received round fits), else folded into the state."""
        if not self.held:
            return
        t = DeviceTable.concat(self.held) if len(self.held) > 1 else self.held[0]
        self.held, self.held_bytes = [], 0
        self.stats["held_batches"] = self.stats.get("held_batches", 0) + 1
        comb = G.combine_partials(t, self.d)
        del t
        if self._state_empty():
            self.direct = comb
            return
        if self.direct is not None:
            prev, self.direct = self.direct, None
            self._fold_in(prev, prev.n)
        self._fold_in(comb, comb.n)

    def _fold_in(self, part: DeviceTable, rows_in: int):
        if self.dense is not None:
            if DenseState.eligible(part) and self.dense.add(part):
                self.stats["dense_state_GB"] = round(self.dense.nbytes() / 1e9, 2)
                return
            # the keys outgrew the dense state: it becomes one piece of the hash-bucket path
            prior, self.dense = self.dense.to_partial(), None
            self.stats["dense_fallback"] = True
            if prior is not None and prior.n:
                self._add_partial(prior, rows_in=rows_in)
        self._add_partial(part, rows_in=rows_in)

    def _add_partial(self, part: DeviceTable, rows_in: int):
        if self.K is None:
            self.p["chunk_bytes_first"] = self.p.get("chunk_bytes_first") or _nbytes(part)
            self._choose_buckets(part, rows_in)
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
        if self.held and self._state_empty():
            # every received partial held: ONE final reduce over them (the bulk stage's kernels)
            t = DeviceTable.concat(self.held) if len(self.held) > 1 else self.held[0]
            self.held, self.held_bytes = [], 0
            self.stats["held_batches"] = self.stats.get("held_batches", 0) + 1
            yield G.final_reduce(t, self.d) if final else G.combine_partials(t, self.d)
            return
        self._flush_held()
        if self.direct is not None and self._state_only_direct():
            t, self.direct = self.direct, None
            yield G.final_reduce(t, self.d) if final else t
            return
        if self.direct is not None:
            t, self.direct = self.direct, None
            self._fold_in(t, t.n)
        if self.dense is not None:
            t = self.dense.to_partial()
            self.dense = None
            if t is not None and t.n:
                yield G.final_reduce(t, self.d) if final else t
            return
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
    out, written = finish(runner, s, p, vctx, agg, final, splan["rest"])
    runner.stream_stats[(s.id, p)] = dict(agg.stats, buckets=agg.K, spilled_buckets=len(agg.spilled),
                                           stream_s=round(t1 - t0, 3),
                                           finish_s=round(time.perf_counter() - t1, 3),
                                           budget_bytes=agg.budget, kind="streamed aggregation",
                                           result=("streamed to the output store" if written is not None
                                                   else "concatenated in HBM"),
                                           result_bytes=written)
    return out


def finish(runner, s, p, vctx, agg: StreamAggregator, final: bool, rest: list):
    """The aggregator's bucket results -> the stage's output value.  A result the stage only
    writes (``rest`` = its output op, a partfile:// or host:// store) goes to the store bucket by
    bucket through runtime/sinks.py, never concatenated in HBM; otherwise the buckets are
    concatenated and the rest of the program runs on them.  Returns (value, bytes streamed or
    None)."""
    from . import sinks
    sink = sinks.for_stage(runner, s, p, rest)
    pending = []
    if sink is not None:
        try:
            for t in agg.bucket_results(final):
                if not pending and sink.add(t):
                    continue
                if sink.started:
                    raise RuntimeError("streamed aggregation: a bucket result could not be written like the others")
                pending.append(t)            # no device encoding: concatenated below
        except BaseException:
            sink.abort()
            raise
        if sink.started:
            value, written = sink.finish()
            return value, written
        pieces = pending
    else:
        pieces = list(agg.bucket_results(final))
    out = DeviceTable.concat(pieces) if pieces else _empty_result(runner, s, vctx, None)
    for op in rest:
        out = runner._run_op(op, [out], vctx, s)
    return out, None


def _empty_result(runner, s, vctx, splan):
    """An empty input partition: the operators' own empty result (host path records nothing)."""
    return []

"""SPMD executor for MI355X ranks: one process per GPU, every rank runs the same plan.

Mapping of the Dryad runtime onto a node of GPUs:
  * vertex placement: partition p of every stage lives on rank ``p % world`` (a GPU "computer");
    pointwise channels between stages are zero-copy hand-offs of HBM tables
  * CrossProduct channels (hash / range shuffles) are one RCCL all-to-all-v of packed rows over
    xGMI per stage; merge / broadcast / remote pointwise channels are gathers / all-gathers
  * the stage DAG executes bulk-synchronously in topological order; the native ``JobGraph``
    tracks vertex versions — a failed vertex is re-executed in place (its inputs are still
    resident in HBM) up to MaxVertexFailures, and a per-stage all-reduce of the status word makes
    every rank abort together instead of hanging in the next collective (gang semantics of
    DrCohort/DrGang: a collective exchange stage restarts as a whole)
  * each op runs as a HIP/PyTorch device op when its lambdas trace to columns (gpu/ops.py);
    otherwise that op alone runs on host objects (recorded in ``self.fallbacks``)
"""
from __future__ import annotations

import atexit
import collections
import json
import os
import pickle
import queue
import threading
import time

import torch
import torch.distributed as dist

from ..compiler.planner import compile_queries
from ..errors import DryadLinqException, DryadLinqJobException, ErrorCode
from ..gpu import ops as G
from ..attributes import is_device_function
from ..gpu.table import DeviceTable, PortTables, Ported, from_objects
from ..gpu.trace import NotTraceable
from ..io.hosttable import HostRows
from ..ops import extsort as EX
from ..io.providers import parse_uri, provider_for
from . import checkpoint as CK
from . import stream_agg as SA
from . import stream_shuffle as SSH
from ..native import runtime as native_runtime
from ..parallel import shuffle
from ..parallel.comm import World, get_world, init_world
from ..utils import trace as TRC
from ..utils.log import get_logger
from . import fused_join as FJ
from . import grace_stage as GS
from . import streaming as ST
from . import vertex_ops as V
from .executor import _BaseExecutor

log = get_logger("gpu_executor")


class ChannelReadError(Exception):
    """A vertex could not read one of its input channels: the producer is blamed (DrGraph.cpp:397-413)."""

    def __init__(self, edge: int, msg: str):
        super().__init__(msg)
        self.edge = edge


class VertexCrash(RuntimeError):
    """A vertex attempt died (its output is discarded and it is re-executed)."""


class VertexCancelled(Exception):
    """A losing speculative attempt stopped at an operator boundary (its duplicate won)."""


class _ColSpec:
    """Vote spec of a columnar fused OrderBy: off -1, length = the packed row bytes."""

    def __init__(self, off: int, length: int):
        self.off, self.length = off, length


class GpuVertexContext(V.VertexContext):
    def __init__(self, partition, partitions, vertex_id, version, stage, device, world, runner=None):
        super().__init__(partition, partitions, vertex_id, version, stage)
        self.device = device
        self.world = world
        self.runner = runner

    def alloc_tensor(self, shape, dtype):
        """Plain device allocation for a vertex's own (non-row) tables."""
        return torch.empty(shape, dtype=dtype, device=self.device)

    def alloc_rows(self, n, stride, layout="plain"):
        """Large row tables come from the executor's HBM pool (reused across jobs).  ``layout``
        "pitch128": the rows live at a 128-byte pitch (a [n, stride] view of [n, 128] rows; only
        for tables that the one-rank fused OrderBy alone reads, see _pitch_gen_reads)."""
        r = self.runner
        if r is None or r.pool is None or self.device.type != "cuda" or n * stride < (64 << 20):
            if layout != "plain":
                return None
            return torch.empty((n, stride), dtype=torch.uint8, device=self.device)
        slack = r.ctx._props.get("ShuffleSlack", 0.01) if self.world.collective else 0.0
        bs = r.pool.acquire(int(n * (1 + slack)) + 1024, stride, layout)
        r.row_sets[(self.stage.id, self.partition)] = bs
        return bs.bufs.rows_in[:n] if layout == "plain" else bs.bufs.rows_in[:n, :stride]


def _to_objects(x):
    if isinstance(x, DeviceTable):
        return x.to_objects()
    if isinstance(x, (Ported, PortTables)):
        return [_to_objects(x.port(k)) for k in range(x.nports)]
    return x


def _object_bytes(x) -> int:
    return x.nbytes if isinstance(x, DeviceTable) else 0


def _device_bytes(x) -> int:
    """HBM bytes behind a vertex input (tables, their string heaps, multi-port outputs)."""
    if isinstance(x, DeviceTable):
        return x.nbytes + (x.heap.numel() if x.heap is not None else 0) + sum(h.numel() for h in x.strs.values())
    if isinstance(x, Ported):
        return _device_bytes(x.table)
    if isinstance(x, PortTables):
        return sum(_device_bytes(t) for t in x.tables)
    return 0


def _records(x) -> int:
    """Records held by an operator argument (a device table, a record list, a ported table)."""
    if x is None:
        return 0
    if isinstance(x, DeviceTable):
        return x.n
    if isinstance(x, Ported):
        return x.table.n
    if isinstance(x, list):
        return sum(_records(y) for y in x) if x and isinstance(x[0], (list, DeviceTable)) else len(x)
    return 1


def _rows100_source(uri) -> bool:
    """gen://terasort, or a stored table of raw 100-byte rows (partfile ``format: rows``)."""
    scheme, path, _ = parse_uri(uri)
    if scheme == "gen":
        return path.strip("/") == "terasort"
    if scheme in ("partfile", "file"):
        try:
            sch = provider_for(uri).schema(uri) or {}
        except Exception:  # noqa: BLE001
            return False
        return sch.get("format") == "rows" and int(sch.get("stride", 0)) == 100
    return False


def _read_sizes(uri, P):
    """Bytes (or rows) of each of the P partitions of a store, known without reading it: the
    partfile metadata's part sizes, or the generator's row ranges (None otherwise)."""
    scheme = parse_uri(uri)[0]
    try:
        if scheme in ("partfile", "file"):
            from ..io import partfile as PF
            m = PF.read_meta(parse_uri(uri)[1])
            return [e.size for e in m.parts] if m.count == P else None
        if scheme == "gen":
            from ..io.providers import GenProvider
            b = [GenProvider().bounds(uri, p) for p in range(P)]
            return [hi - lo for lo, hi in b]
    except Exception:  # noqa: BLE001
        return None
    return None


class GpuJobRunner:
    def __init__(self, ctx, plan, world: World, faults=None, pool=None):
        self.ctx, self.plan, self.world = ctx, plan, world
        self.pool = pool
        self.row_sets: dict = {}          # (stage, partition) -> pooled BufferSet holding its rows
        self.moved: dict = {}             # (stage, partition) -> rank whose duplicate attempt won
        self.stream_plans: dict = {}      # stage -> chunk plan of a streamed stage (None: not streamed)
        self.agg_plans: dict = {}         # stage -> plan of a streamed (out-of-core) GroupBy / Distinct
        self.part_stream_plans: dict = {}  # stage -> plan of a streamed HashPartition -> ToStore
        self.empty_host_ops: list = []    # host operators that ran over empty inputs only
        self.stream_stats: dict = {}      # (stage, partition) -> chunks / records / bytes streamed
        self.place = None                 # partition -> rank (None: p % W)
        self.fused: dict = {}             # merge stage id -> fused distributed-OrderBy descriptor
        self.skipped: set = set()
        self.dev = world.device
        self.gpu_ok = self.dev.type == "cuda"
        self.faults = faults or []
        self.channels: dict = {}          # (stage, partition) -> DeviceTable | Ported | list | list-of-lists
        self.fallbacks: list = []
        self.op_counts = collections.Counter()   # (operator, "device" | "host") -> executions
        from ..io.writer import WriteStats
        self.write_stats = WriteStats()          # partfile parts written by this job
        self.recycled_parts = 0                  # of them, recycled parts of a replaced table
        self.phases: dict = {}                   # host seconds: setup / stages / commit (run_job: compile, total)
        from ..io.reader import ReadStats
        self.read_stats = ReadStats()            # part files read into HBM by this job
        self.transports: list = []      # (stage, edge kind, "device" | "object", bytes / reason)
        self.timings: dict = {}
        R = native_runtime()
        p = R.Params()
        p.max_failures = int(getattr(ctx, "MaxVertexFailures", 6) or 6)
        # speculative duplicates (DrDefaultManager::CheckForDuplicates) only for leaf stages outside
        # gangs: a duplicate re-reads the vertex's source on an idle rank (no collective inside).
        # On one node of identical GPUs the reference's adaptive threshold (>= 10 s,
        # DrStageStatistics.cpp:93-111) almost never fires, while the speculative stage loop polls
        # a collective every SPEC_POLL behind the vertices' kernels: the GPU executor speculates
        # only under an explicit straggler policy (OutlierThresholdSeconds set).
        thr = ctx._props.get("OutlierThresholdSeconds")
        p.speculative = bool(getattr(ctx, "EnableSpeculativeDuplication", True)) and world.size > 1 \
            and thr is not None
        if thr is not None:
            p.default_outlier_threshold = float(thr)
            p.min_outlier_threshold = min(p.min_outlier_threshold, float(thr))
        self.g = R.JobGraph(p)
        self.g_speculative = p.speculative
        self.vids = []
        self.part_of, self.stage_of = {}, {}
        for s in plan.stages:
            self.g.add_stage(f"{s.id}:{s.name}", s.partitions, p.speculative and self._duplicable(s, plan), s.is_output)
            self.vids.append([self.g.add_vertex(s.id, q) for q in range(s.partitions)])
            for q, v in enumerate(self.vids[-1]):
                self.part_of[v], self.stage_of[v] = q, s.id
        self.edge_ids = {}               # (src vertex, dst vertex, input) -> JobGraph edge id
        for s in plan.stages:
            for q in range(s.partitions):
                for ii, si in enumerate(s.inputs):
                    for src in self._sources(si, q):
                        self.edge_ids[(self.vids[si.src][src], self.vids[s.id][q], ii)] = len(self.edge_ids)
                        self.g.add_edge(self.vids[si.src][src], 0, self.vids[s.id][q], ii)
        # gangs (DrGang, DrCohort.cpp:852): the members of one collective exchange restart together
        self.gang_stages = set()
        for s in plan.stages:
            if any(si.kind == "cross" for si in s.inputs) and s.partitions > 1:
                self.g.set_gang(self.vids[s.id])
                self.gang_stages.add(s.id)
        self.recovery: list = []         # recovery actions taken (tests / statistics)
        self.ckpt = None                 # runtime/checkpoint.StageCheckpoint of a resumable job
        self.persist_stats: dict = {}    # stage name -> persisted bytes / ms (or why it was not)
        self.persist_seconds = 0.0
        self.precomputed_bodies: dict = {}   # fused join stage id -> (attempt body, program after it)

    @staticmethod
    def _duplicable(s, plan) -> bool:
        """A stage whose vertices a duplicate can run anywhere: no input channels (it reads its
        source itself, re-readable: the reference's inputs are immutable files too)."""
        if s.inputs or not s.ops:
            return False
        o = s.ops[0]
        return o["op"] == "enumerable" or (o["op"] == "read" and parse_uri(o["uri"])[0] in ("gen", "partfile", "file"))

    def owner(self, p: int, sid: int | None = None) -> int:
        """Rank of partition p (of stage ``sid``): a speculative duplicate that won moved that one
        vertex's output (``moved``); otherwise the job's placement (``place``, by input size when
        there are more partitions than ranks), else p % W."""
        if sid is not None and self.moved and (sid, p) in self.moved:
            return self.moved[(sid, p)]
        if self.place is not None and p < len(self.place):
            return self.place[p]
        return p % self.world.size

    # ------------------------------------------------------------------ placement
    def _placement(self):
        """Partition -> rank when the job has more partitions than ranks.  The reference places each
        vertex by its inputs' location and size (LocalScheduler.ScheduleProcessInternal,
        LocalScheduler.cs:132-268; the GM passes input size hints, DrVertex.cpp:356-429); here the
        partitions of the job's largest leaf read (sizes from the partfile metadata or the
        generator's ranges, the same on every rank) go largest first to the least-loaded rank, and
        every stage keeps that map, so pointwise channels stay local.  None (p % W) when the job
        has no more partitions than ranks or the sizes are unknown / equal."""
        W = self.world.size
        P = max((st.partitions for st in self.plan.stages), default=1)
        if W == 1 or P <= W:
            return None
        best = None
        for st in self.plan.stages:
            if st.inputs or st.partitions != P or not st.ops or st.ops[0]["op"] != "read":
                continue
            sizes = _read_sizes(st.ops[0]["uri"], P)
            if sizes is not None and (best is None or sum(sizes) > sum(best)):
                best = sizes
        if best is None or len(set(best)) == 1:
            return None
        load, place = [0] * W, [0] * P
        for p in sorted(range(P), key=lambda q: (-best[q], q)):
            r = min(range(W), key=lambda k: (load[k], k))
            place[p] = r
            load[r] += best[p]
        return place

    # ------------------------------------------------------------------ fused distributed OrderBy
    def _find_fused_orderby(self):
        """Plan idiom Sample -> Separators -> RangePartition -(cross)-> Merge+sort over one input X.
        For fixed-width row tables it runs as ONE gang stage: the pooled in-place distributed sort
        (ops/recordsort.distributed_sort_rows) with no intermediate table copies."""
        st = self.plan.stages
        out = {}
        for m in st:
            if len(m.inputs) != 1 or m.inputs[0].kind != "cross" or not m.ops or m.ops[0]["op"] != "sort":
                continue
            rp = st[m.inputs[0].src]
            if len(rp.ops) != 1 or rp.ops[0]["op"] != "range_partition" or rp.ops[0].get("separators") is not None:
                continue
            if len(rp.inputs) != 2 or rp.inputs[0].kind != "pointwise" or rp.inputs[1].kind != "broadcast":
                continue
            sep = st[rp.inputs[1].src]
            if len(sep.inputs) != 1 or sep.inputs[0].kind != "merge" or sep.ops[0]["op"] != "separators":
                continue
            samp = st[sep.inputs[0].src]
            x = rp.inputs[0].src
            if len(samp.inputs) != 1 or samp.inputs[0].src != x or samp.ops[0]["op"] != "sample" or len(samp.ops) != 1:
                continue
            if self.plan.consumers(samp.id) != [sep.id] or self.plan.consumers(sep.id) != [rp.id] or \
                    self.plan.consumers(rp.id) != [m.id]:
                continue
            if rp.partitions != st[x].partitions or m.partitions != st[x].partitions:
                continue
            out[m.id] = dict(x=x, stages=[samp.id, sep.id, rp.id], key=m.ops[0]["key"],
                             desc=m.ops[0].get("descending", False), comparer=m.ops[0].get("comparer"),
                             keep_ties=bool(rp.ops[0].get("keep_ties", False)))
        return out

    def _fused_applicable(self, f) -> bool:
        from ..gpu import trace as TR
        from ..ops import rowpack as RP
        colvals = []
        ok = self.gpu_ok and f["comparer"] is None and self.plan.stages[f["x"]].partitions == self.world.size
        spec = None
        if ok:
            t = self.channels.get((f["x"], self.world.rank))
            # a table in a pooled buffer set is sorted in place; any other row table (an hbm://
            # input, a previous job's output) is read where it is, into a set of its own
            ok = isinstance(t, DeviceTable) and t.rows is not None and (
                (f["x"], self.world.rank) in self.row_sets or (self.pool is not None and t.rows.is_contiguous()))
            if ok:
                try:
                    kind, spec = TR.key_columns(TR.call(f["key"], t), t)
                    ok = kind == "bytes" and spec.length <= 12
                except Exception:  # noqa: BLE001
                    ok = False
                if not ok:
                    spec = None
            elif isinstance(t, DeviceTable) and t.rows is None and self.pool is not None:
                # a columnar table with numeric key parts: packed into byte-keyed rows
                # (ops/rowpack.py) for the same exchange, each part cut to the job's value range
                # (the bounds travel in the vote); spec (-1, key parts)
                try:
                    kind, keys = TR.key_columns(TR.call(f["key"], t), t)
                    pre = RP.plan(t, keys, [(0, 0)] * len(keys)) \
                        if kind == "cols" and len(keys) <= RP.MAX_KEY_BYTES else None
                    if pre is not None:
                        colvals = RP.key_bounds(keys, t.n)
                except Exception:  # noqa: BLE001
                    pre = None
                if pre is not None:
                    ok = True
                    spec = _ColSpec(-1, len(keys))
        mine = None if spec is None else (spec.off, spec.length)
        pad = list(colvals) + [(1 << 63) - 1, -(1 << 63)] * RP.MAX_KEY_BYTES
        agree, vals = shuffle.vote(bool(ok), mine, self.world, values=pad[: 2 * RP.MAX_KEY_BYTES])
        if agree and mine is not None and mine[0] < 0:
            f["colbounds"] = RP.merge_bounds(vals, mine[1])
            lay = RP.plan(t, keys, f["colbounds"])         # the same decision on every rank
            if lay is None:
                return False
            mine = (-1, lay.rec)
        if agree:
            f["spec"] = mine
            return True
        return False

    def _lazy_gen_reads(self) -> set:
        """gen://terasort read stages whose table only a fused distributed OrderBy consumes: their
        op_read writes just the sort entries (ops/gpu: lazy_gen) and the records are generated
        straight into the exchange's send buckets."""
        st, out = self.plan.stages, set()
        if not self.world.collective or not self.gpu_ok or not self.ctx._props.get("GenFusedShuffle", False):
            return out
        for f in self.fused.values():
            x = st[f["x"]]
            if (not x.inputs and len(x.ops) == 1 and x.ops[0]["op"] == "read"
                    and parse_uri(x.ops[0]["uri"])[0] == "gen" and parse_uri(x.ops[0]["uri"])[1].strip("/") == "terasort"
                    and set(self.plan.consumers(x.id)) == {f["stages"][0], f["stages"][2]}):
                out.add(x.id)
        return out

    def _pitch_gen_reads(self) -> dict:
        """One rank: stages ``read(100-byte records) -> sort(ascending byte-string key of <= 16
        bytes) -> ...`` (the one-rank OrderBy plan) over gen://terasort or a stored table of raw
        100-byte rows (partfile ``format: rows``).  Their op_read stores the records at a 128-byte
        pitch (one aligned HBM line per record) and op_sort sorts them with
        ops/sort.sort_rows_pitch128: the sort's random row reads fetch one line per record
        instead of ~1.78.  ``LineAlignedSortInput=False`` (context property) turns it off.
        Returns {stage id: (key offset, key length)}."""
        out = {}
        if not self.gpu_ok or not self.ctx._props.get("LineAlignedSortInput", True):
            return out
        from ..gpu import trace as TR
        from ..gpu.table import Shape
        if self.world.collective:
            return self._pitch_fused_reads()
        for x in self.plan.stages:
            if not (not x.inputs and len(x.ops) >= 2 and x.ops[0]["op"] == "read" and x.ops[1]["op"] == "sort"
                    and _rows100_source(x.ops[0]["uri"])
                    and x.ops[1].get("comparer") is None and not x.ops[1].get("descending", False)):
                continue
            rows = torch.zeros((2, 100), dtype=torch.uint8, device=self.dev)
            t = DeviceTable(2, Shape("rows", key_off=0, key_len=10), rows=rows)
            try:
                kind, spec = TR.key_columns(TR.call(x.ops[1]["key"], t), t)
            except Exception:  # noqa: BLE001
                continue
            if kind == "bytes" and 1 <= spec.length <= 16 and spec.off + spec.length <= 100:
                out[x.id] = (spec.off, spec.length)
        return out

    def _pitch_fused_reads(self) -> dict:
        """Several ranks: read stages of 100-byte rows (gen://terasort or a stored ``format: rows``
        table) that only a fused distributed OrderBy on key bytes 0..9 consumes.  Their op_read
        stores the records at a 128-byte pitch with the E64 entries (+ window histograms) in the
        send buffer's memory, and the fused stage runs the fine-bucket exchange over that table
        (ops/recordsort.send_fine_rows: the send-side row gather reads one HBM line per record).
        ``GenFusedShuffle`` keeps gen:// reads lazy instead (records generated into the send rows)."""
        from ..gpu import trace as TR
        from ..gpu.table import Shape
        from ..ops import recordsort as RS
        st, out = self.plan.stages, {}
        lazy = self._lazy_gen_reads()
        for f in self.fused.values():
            x = st[f["x"]]
            if (x.id in lazy or x.inputs or len(x.ops) != 1 or x.ops[0]["op"] != "read"
                    or not _rows100_source(x.ops[0]["uri"]) or f["comparer"] is not None or f["desc"]
                    or set(self.plan.consumers(x.id)) != {f["stages"][0], f["stages"][2]}
                    or not RS.fine_rows_ok(100, 128, 0, 10, self.world.size, 1, self.world.force_collectives)):
                continue
            rows = torch.zeros((2, 100), dtype=torch.uint8, device=self.dev)
            t = DeviceTable(2, Shape("rows", key_off=0, key_len=10), rows=rows)
            try:
                kind, spec = TR.key_columns(TR.call(f["key"], t), t)
            except Exception:  # noqa: BLE001
                continue
            if kind == "bytes" and spec.off == 0 and spec.length == 10:
                out[x.id] = (0, 10)
        return out

    def _materialize(self, sid: int):
        """Write the records of lazy gen reads of stage sid (its consumers are not fused after all)."""
        for p in range(self.plan.stages[sid].partitions):
            bs = self.row_sets.get((sid, p))
            t = self.channels.get((sid, p))
            if bs is not None and bs.lazy_gen is not None and isinstance(t, DeviceTable):
                bs.materialize(t.n)


    def _run_fused(self, m, f):
        from ..ops import recordsort as RS
        me = self.world.rank
        t = self.channels[(f["x"], me)]
        bs = self.row_sets.get((f["x"], me))
        off, ln = f["spec"]
        stats = RS.SortStats()
        src = None
        if off < 0:
            return self._run_fused_columns(m, f, t, stats)
        if bs is None:
            # the input table is not ours to clobber: its rows are read in place (entries, the
            # send-side pack) and the exchange works in a buffer set of its own
            slack = self.ctx._props.get("ShuffleSlack", 0.01)
            bs = self.pool.acquire(int(t.n * (1 + slack)) + 1024, t.rows.shape[1])
            src = t.rows
            kr, gen = None, None
        else:
            f["consumed"] = (bs.lazy_gen, bs.keys_ready)      # what a retry restores (gen inputs)
            kr = bs.take_keys(t.rows, off, ln)
            gen, bs.lazy_gen = bs.lazy_gen, None
            f["clobbered"] = True                             # rows_in becomes the receive buffer
            if gen is not None and kr is None:         # entries were not claimed: records are needed
                bs.lazy_gen = gen
                bs.materialize(t.n)
                gen = None
        out = RS.distributed_sort_rows(bs.bufs, t.n, off, ln, self.world, stats=stats,
                                       keys_ready=kr is not None, hi_bounds=None if kr is None else kr[:2],
                                       split_ties=not f.get("keep_ties", False),
                                       keys_fmt="e128" if kr is None else kr[2], gen=gen, src=src,
                                       descending=bool(f.get("desc", False)))
        self.row_sets[(m.id, me)] = bs
        self.last_sort_stats = stats
        table = DeviceTable(out.shape[0], t.shape, rows=out)
        # the rest of the merge stage's program after the sort
        vctx = GpuVertexContext(me, m.partitions, self.vids[m.id][me], 0, m, self.dev, self.world, self)
        data = table
        for op in m.ops[1:]:
            data = self._run_op(op, [data], vctx, m)
        return data

    def _run_fused_columns(self, m, f, t, stats):
        """The fused OrderBy of a columnar table: its rows packed with the byte-comparable key
        first into a buffer set of their own (the input stays intact), the fine-bucket exchange,
        the received rows unpacked into columns that live in the set's input memory (free once
        the exchange has merged every round)."""
        from ..gpu import trace as TR
        from ..ops import recordsort as RS
        from ..ops import rowpack as RP
        me = self.world.rank
        _, keys = TR.key_columns(TR.call(f["key"], t), t)
        lay = RP.plan(t, keys, f["colbounds"])
        if lay is None or lay.rec != f["spec"][1]:
            raise RuntimeError("fused columnar OrderBy: the row layout changed after the vote")
        slack = self.ctx._props.get("ShuffleSlack", 0.01)
        bs = self.pool.acquire(int(t.n * (1 + slack)) + 1024, lay.rec)
        RP.pack(t, keys, lay, bs.bufs.rows_in[: t.n])
        out = RS.distributed_sort_rows(bs.bufs, t.n, 0, lay.key_len, self.world, stats=stats,
                                       split_ties=not f.get("keep_ties", False),
                                       descending=bool(f.get("desc", False)))
        mem = bs.bufs.rows_in.view(-1) if out.data_ptr() == bs.bufs.rows_out.data_ptr() else None
        cols = RP.unpack(out, lay, mem)
        stats.path = f"columns packed into {lay.rec}-byte rows, " + (stats.path or "")
        self.row_sets[(m.id, me)] = bs
        self.last_sort_stats = stats
        vctx = GpuVertexContext(me, m.partitions, self.vids[m.id][me], 0, m, self.dev, self.world, self)
        data = DeviceTable(out.shape[0], t.shape, cols)
        for op in m.ops[1:]:
            data = self._run_op(op, [data], vctx, m)
        return data

    # ------------------------------------------------------------------ fused gang stages
    def _run_gang(self, s, body, ready, refresh, now, restore=None):
        """Run a fused stage (distributed or out-of-core OrderBy) as versioned attempts of its
        vertices, the reference's gang re-execution (DrGang::EnsurePendingVersion, DrCohort.cpp:852;
        DrActiveVertex::ReactToFailedVertex, DrVertex.cpp:1042-1171; DrGraph::ReportFailure,
        DrGraph.cpp:392-456).  One attempt = ``body()`` on every rank (it holds collectives).

        Decisions are voted so no rank enters a collective alone: injected faults are agreed
        before the body (fail, read_error, slow) and after it (crash: the attempt's output is
        discarded), and each rank's outcome after it.  A failed attempt fails the vertex of its
        rank's partition, and every member restarts at its next version (gang) after ``restore()``
        rebuilt what the attempt consumed; a read error re-reads the input from lineage first.
        MaxVertexFailures failures abort the job.  An exception raised inside the collective body
        on one rank only leaves its peers in the exchange: the communicator's error handling then
        ends the job (parallel/comm.py), as a lost process would."""
        g, W, me = self.g, self.world.size, self.world.rank
        mine = [p for p in range(s.partitions) if self.owner(p, s.id) == me]
        while True:
            refresh()
            vers = {}
            for p in range(s.partitions):
                vid = self.vids[s.id][p]
                vers[p] = ready.pop(vid)
                g.on_running(vid, vers[p], self.owner(p, s.id), now())
            faults = {p: self._fault(s, p, vers[p]) for p in mine}
            pre = next(((p, k) for p, k in faults.items() if k in ("fail", "read_error")), None)
            for k in faults.values():
                if k and k.startswith("slow"):
                    time.sleep(float(k.split(":")[1]) if ":" in k else 1.0)
            outcome = self._vote(None if pre is None else (pre[0], pre[1], f"injected {pre[1]} of {s.name}[{pre[0]}]"))
            out = None
            if outcome is None:
                err = None
                try:
                    out = body()
                    crash = next((p for p, k in faults.items() if k == "crash"), None)
                    if crash is not None:
                        err = (crash, "crash", f"injected crash of {s.name}[{crash}] (output discarded)")
                except Exception as e:  # noqa: BLE001
                    self._last_exc = e
                    # a deterministic failure every rank agreed on before the exchange (range
                    # skew past capacity): re-executing would fail alike, so the job ends now
                    kind = "fatal" if getattr(e, "retryable", True) is False else "fail"
                    err = (mine[0] if mine else 0, kind, f"{type(e).__name__}: {e}")
                outcome = self._vote(err)
            if outcome is None:
                for p in range(s.partitions):
                    g.on_completed(self.vids[s.id][p], vers[p], now(), 0, _object_bytes(out) if p in mine else 0)
                return out
            failed = {}
            for r, (p, kind, msg) in outcome:
                failed[p] = (kind, msg)
                self._dump_restart(s, p, vers[p], [], msg) if r == me else None
                log.warning("fused stage %s[%d] v%d failed (%s): %s", s.name, p, vers[p], kind, msg)
            for p in sorted(failed):                # the first failure restarts the whole gang
                g.on_failed(self.vids[s.id][p], vers[p], now(), -1, failed[p][1])
                self.recovery.append(("upstream" if failed[p][0] == "read_error" else "gang_restart", s.name, p))
            fatal = [msg for kind, msg in failed.values() if kind == "fatal"]
            if fatal:
                raise DryadLinqJobException(ErrorCode.JobToCreateTableFailed, f"{s.name}: {fatal[0]}",
                                            inner=getattr(self, "_last_exc", None))
            if g.failed():
                raise DryadLinqJobException(ErrorCode.JobToCreateTableFailed, g.failure(),
                                            inner=getattr(self, "_last_exc", None))
            if restore is not None:
                restore(any(k == "read_error" for k, _ in failed.values()))

    def _vote(self, err):
        """All-gather of each rank's attempt outcome: None (ok) or (partition, kind, message).
        Returns None when every rank succeeded, else [(rank, outcome)] of the failures."""
        got = self._gather_if_any(err) if self.world.size > 1 else ([err] if err is not None else None)
        if got is None:
            return None
        bad = [(r, e) for r, e in enumerate(got) if e is not None]
        return bad or None

    def _gather_if_any(self, obj):
        """None when every rank passes None (one tensor all-gather of a flag, no pickling: the
        per-stage votes of an iterative job stay off the host's object path), else every rank's
        record (JSON over a tensor all-gather, only when some rank has something to say)."""
        from ..parallel import shuffle
        st = shuffle.gang_status(obj is None, 0, self.world)
        if all(ok for ok, _ in st):
            return None
        return self._gather_objects(obj)

    def _gather_objects(self, obj):
        """Every rank's outcome records (ints, strings), as JSON over a tensor all-gather."""
        return shuffle.gather_json(obj, self.world)

    def _restore_fused_input(self, f, reread: bool = False):
        """Before a retry of a fused distributed OrderBy: its input table again.  A gen://terasort
        input that was never written only needs its generator parameters back; a table the
        failed attempt clobbered (rows_in became the receive buffer), or one whose read failed
        (``reread``), is rebuilt from lineage.  Collective (every rank decides alike: the
        outcome was voted)."""
        me = self.world.rank
        clobbered = f.pop("clobbered", False)
        bs = self.row_sets.get((f["x"], me))
        gen, keys = f.pop("consumed", (None, None)) if clobbered else (bs.lazy_gen if bs else None, None)
        if bs is not None and gen is not None:
            if clobbered:
                bs.lazy_gen, bs.keys_ready = gen, keys
            return
        if not clobbered and not reread:
            return
        if bs is not None and self.pool is not None:
            self.pool.release(bs)               # the rebuilt table reuses the same HBM
        for key in [k for k in self.channels if k[0] == f["x"]]:
            del self.channels[key]
        self._rematerialize(f["x"])

    # ------------------------------------------------------------------ out-of-core OrderBy
    def _plan_external(self):
        """OrderBy jobs whose partitions do not fit the HBM budget: ``read -> sort -> output`` (one
        partition per rank) or the distributed idiom over such a read, writing a ``host://``
        table.  They run as ops/extsort.external_sort, streaming the source through HBM in chunks
        and spilling range buckets to pinned host memory (the reference's ParallelSort spill,
        DryadLinqVertex.cs:9584-9615).  ``ExternalSort`` (context property) forces (True) or
        forbids (False) the path; otherwise it is taken when rows in + out + entries would exceed
        ``HbmBudgetBytes`` (default 80% of free HBM)."""
        props = self.ctx._props
        force = props.get("ExternalSort")
        if force is False or not self.gpu_ok:
            return {}
        st, W = self.plan.stages, self.world.size
        cands = {}
        for s in st:
            if (not s.inputs and len(s.ops) >= 2 and s.ops[0]["op"] == "read" and s.ops[1]["op"] == "sort"
                    and all(op["op"] == "output" for op in s.ops[2:]) and s.is_output and s.partitions == W):
                cands[s.id] = dict(read=s.ops[0], sort=s.ops[1], skip=[], keep_ties=False)
        for mid, f in self.fused.items():
            m, x = st[mid], st[f["x"]]
            if (not x.inputs and len(x.ops) == 1 and x.ops[0]["op"] == "read" and m.is_output
                    and all(op["op"] == "output" for op in m.ops[1:]) and x.partitions == W
                    and set(self.plan.consumers(x.id)) == {f["stages"][0], f["stages"][2]}):
                cands[mid] = dict(read=x.ops[0], sort=m.ops[0], skip=[x.id] + f["stages"], keep_ties=f["keep_ties"])
        out = {}
        for sid, c in sorted(cands.items()):
            sort = c["sort"]
            ok = parse_uri(st[sid].output["uri"])[0] in ("host", "partfile", "file") and sort.get("comparer") is None
            src = self._chunk_source(c["read"]) if ok else None
            spec = None
            if src is not None:
                spec = self._external_key(src, c["read"], sort["key"])
                budget = props.get("HbmBudgetBytes")
                need = src.n * (2 * src.stride + 32) * 1.05
                ok = spec is not None and (force is True or need > int(budget or EX.default_budget(self.dev)))
            else:
                ok = False
            agree, _ = shuffle.vote(bool(ok), spec, self.world)
            if agree:
                out[sid] = dict(c, source=src, spec=spec)
        return out

    def _chunk_source(self, op):
        uri = op["uri"]
        scheme, path, q = parse_uri(uri)
        me = self.world.rank
        if scheme == "gen" and path.strip("/") == "terasort":
            from ..io.providers import GenProvider
            lo, hi = GenProvider().bounds(uri, me)
            return EX.GenTeraSortSource(lo, hi - lo, int(q.get("seed", 0)))
        if scheme == "host":
            prov = provider_for(uri)
            h = prov.local_rows(uri, me) if prov.exists(uri) else None
            return EX.HostRowsSource(h) if h is not None and h.stride % 4 == 0 else None
        if scheme in ("partfile", "file"):
            prov = provider_for(uri)
            r = prov.rows_part(uri, me) if prov.exists(uri) else None
            return EX.MappedRowsSource(*r) if r is not None and r[0].shape[1] % 4 == 0 else None
        return None

    def _external_key(self, src, read_op, key):
        """(key offset, key length) of a byte-string key selector over the source's rows."""
        from ..gpu import trace as TR
        from ..gpu.table import Shape
        k = max(1, min(src.n, 2))
        rows = torch.zeros((k, src.stride), dtype=torch.uint8, device=self.dev)
        if src.n:
            src.fill(0, k, rows, None)
        ko, kl = getattr(src, "key_spec", (0, 10))
        shape = Shape("rows", key_off=ko, key_len=kl)
        try:
            kind, spec = TR.key_columns(TR.call(key, DeviceTable(k, shape, rows=rows)), DeviceTable(k, shape, rows=rows))
        except Exception:  # noqa: BLE001
            return None
        return (spec.off, spec.length) if kind == "bytes" and spec.length <= 12 else None

    def _run_external(self, s, e):
        if self.pool is not None:
            self.pool.clear()           # idle pooled sort buffers give their HBM back
            torch.cuda.empty_cache()
        off, ln = e["spec"]
        st = EX.ExtSortStats()
        factory = self._disk_output(s, e["source"], off, ln)
        out = EX.external_sort(e["source"], off, ln, self.world, budget=self.ctx._props.get("HbmBudgetBytes"),
                               keep_ties=e["keep_ties"], stats=st, out_factory=factory,
                               descending=bool(e["sort"].get("descending", False)))
        self.extsort_stats = st
        return out

    def _disk_output(self, s, src, off, ln):
        """Disk tier for an out-of-core OrderBy writing ``partfile://``: a factory that places this
        rank's sorted rows in a memory-mapped file next to the output (renamed into the part file
        at commit), so the output need not fit host memory.  ``ExternalSortToDisk`` forces / forbids
        it; by default it is used when the rank's output would take over half the available RAM."""
        scheme, path, _ = parse_uri(s.output["uri"])
        if scheme not in ("partfile", "file"):
            return None
        force = self.ctx._props.get("ExternalSortToDisk")
        if force is False:
            return None
        if force is None:
            import psutil
            if src.n * src.stride * 1.1 < 0.5 * psutil.virtual_memory().available:
                return None
        tmp = f"{os.path.abspath(path)}.extsort.{self.world.rank}.{os.getpid()}.tmp"
        os.makedirs(os.path.dirname(tmp) or ".", exist_ok=True)
        return lambda n_out: HostRows.mapped(tmp, n_out, src.stride, off, ln)

    def _sources(self, si, p):
        src = self.plan.stages[si.src]
        if si.kind == "pointwise":
            return [p]
        if si.kind == "offset":
            q = p - si.offset
            return [q] if 0 <= q < src.partitions else []
        if si.kind == "group":
            return list(range(p * si.group, min(src.partitions, (p + 1) * si.group)))
        return list(range(src.partitions))

    def _combine_local(self, s, si, parts):
        """One partial folding this rank's partials of the source stage (agg_combine)."""
        vals = [self._port_of(si, self.channels[(si.src, q)], None) for q in parts]
        vals = [_to_objects(v) if not isinstance(v, list) else v for v in vals]
        vctx = GpuVertexContext(0, 1, -1, 0, s, self.dev, self.world, self)
        return V.OPS["agg_combine"](dict(op="agg_combine", spec=s.ops[0]["spec"]), [[x for v in vals for x in v]],
                                    vctx)

    # ------------------------------------------------------------------ channel transport
    def _port_of(self, si, val, dst_p):
        """Port data of one source vertex's output for a destination partition."""
        if si.kind == "cross":
            if isinstance(val, Ported):
                return val.port(dst_p)
            return val[dst_p]
        k = si.port
        if isinstance(val, (Ported, PortTables)):
            return val.port(k)
        if isinstance(val, list) and val and isinstance(val[0], list) and self.plan.stages[si.src].out_ports > 1:
            return val[k]
        return val

    def _gather_inputs(self, s, only=None, recover=False):
        """Deliver every input channel of every local vertex of stage s (collectives included);
        ``only``: just these partitions (re-execution).  Source channels released after an earlier
        delivery are rebuilt from lineage first (all ranks release in lockstep)."""
        W, me = self.world.size, self.world.rank
        local = [p for p in range(s.partitions) if self.owner(p, s.id) == me and (only is None or p in only)]
        inputs = {p: [[] for _ in s.inputs] for p in local}
        for ii, si in enumerate(s.inputs):
            src_stage = self.plan.stages[si.src]
            so = lambda q, _s=si.src: self.owner(q, _s)  # noqa: E731  (source partition -> its rank)
            do = lambda p, _s=s.id: self.owner(p, _s)    # noqa: E731
            if recover:      # (collective vote: a rank that owns no source partition still takes part)
                mine = [q for q in range(src_stage.partitions) if so(q) == me]
                lost = any((si.src, q) not in self.channels for q in mine)
                miss = [not ok for ok, _ in shuffle.gang_status(not lost, 0, self.world)] if W > 1 else [lost]
                if any(miss):
                    self._rematerialize(si.src)
            if si.kind == "cross" and W > 1:
                got = self._exchange_cross(si, src_stage, s)
                for p in local:
                    inputs[p][ii] = got[p]
                continue
            # which (src q -> dst p) items cross ranks?
            dst_parts = range(s.partitions) if only is None else only
            need_remote = False
            for p in dst_parts:
                for q in self._sources(si, p):
                    if so(q) != do(p):
                        need_remote = True
            if not need_remote:
                for p in local:
                    inputs[p][ii] = [self._port_of(si, self.channels[(si.src, q)], p) for q in self._sources(si, p)]
                continue
            if si.kind == "merge" and s.dynamic_manager == "FullAggregator" and only is None \
                    and s.ops and s.ops[0]["op"] == "agg_final":
                # dynamic aggregation level 1 (DrDynamicAggregateManager machine grouping): each rank
                # folds the partials of its own source partitions into one before the final vertex
                mine = [q for q in range(src_stage.partitions) if so(q) == me]
                got = self._transport(s, si, [[self._combine_local(s, si, mine)] if do(0) == r else []
                                              for r in range(W)],
                                      [[("rank", r)] if do(0) == me else [] for r in range(W)])
                for p in local:
                    inputs[p][ii] = [x for r in range(W) for x in got[r].values()]
                self.recovery.append(("dynamic_aggregate", s.name, len(mine)))
                continue
            # merge / broadcast / remote pointwise edges: every rank sends each port value another
            # rank needs once (a q feeding several of its partitions travels once)
            need = [sorted({q for p in dst_parts if do(p) == r for q in self._sources(si, p)
                            if so(q) != r}) for r in range(W)]
            mine = {q: self._port_of(si, self.channels[(si.src, q)], None) for r in range(W) for q in need[r]
                    if so(q) == me}
            sends = [[mine[q] for q in need[r] if so(q) == me] for r in range(W)]
            got = self._transport(s, si, sends, [[q for q in need[me] if so(q) == r] for r in range(W)])
            recv = {q: x for r in range(W) for q, x in got[r].items()}
            for p in local:
                inputs[p][ii] = [self._port_of(si, self.channels[(si.src, q)], p) if so(q) == me
                                 else recv[q] for q in self._sources(si, p)]
        return inputs

    # ------------------------------------------------------------------ channel transport
    def _transport(self, s, si, sends, recv_ids):
        """Move port values between ranks: ``sends[r]`` = values for rank r (in ``recv_ids`` order on
        the receiving side), through the first transport of the channel registry
        (parallel/channels.py) every rank can use: device tables of one schema as RCCL
        all-to-all-v per column (string heaps included), anything else as host objects, recorded
        in ``self.transports``.  Returns, per source rank, {source partition: value}."""
        from ..parallel import channels as CHN
        from ..parallel import exchange as EXC
        W = self.world.size
        why = None
        for tr in CHN.transports():
            ok = tr.usable(sends)
            from ..parallel import shuffle as SH
            if not all(v for v, _ in SH.gang_status(bool(ok), 0, self.world)):
                why = why or ("host records on the channel" if tr.name == "device" else f"{tr.name} not usable")
                continue
            try:
                got, kind, detail = tr.move(self, sends)
            except EXC.SchemaMismatch as e:
                why = str(e)
                continue
            if kind == "scalar" and why and why.startswith("ranks"):
                kind = "object"          # the ranks' tables disagree: not a control-plane partial
            self.transports.append((s.name, si.kind, kind, detail if kind == "device" or why is None else why))
            return [dict(zip(recv_ids[r], got[r])) for r in range(W)]
        raise RuntimeError("no channel transport could move the values")

    @staticmethod
    def _ship(x):
        """A port for the object transport: string-bearing device tables travel as host copies of
        their columns and heaps (so field names, partial-aggregate layouts and the device path on
        the receiving rank survive); everything else as records."""
        if isinstance(x, DeviceTable) and (x.heap is not None or x.strs):
            return ("dts", x.shape, {k: v.cpu() for k, v in x.cols.items()},
                    x.heap.cpu() if x.heap is not None else None, {f: h.cpu() for f, h in x.strs.items()}, x.n)
        return ("obj", _to_objects(x))

    def _unship(self, x):
        if x[0] == "dts":
            _, shape, cols, heap, strs, n = x
            return DeviceTable(n, shape, {k: v.to(self.dev) for k, v in cols.items()},
                               heap=heap.to(self.dev) if heap is not None else None,
                               strs={f: h.to(self.dev) for f, h in strs.items()})
        return x[1]

    def _exchange_cross(self, si, src_stage, dst_stage):
        """CrossProduct shuffle (HashPartition/RangePartition -> Merge): ONE exchange of the port
        slices.  Send order per destination rank: local source partitions ascending, then that
        rank's partitions ascending; with one partition per rank and rank-major port order
        (gpu/ops.partition_by_entries) each rank's pieces are one slice of the producer's columns
        and the pieces a partition receives arrive adjacent, so neither side copies."""
        W, me = self.world.size, self.world.rank
        P_src, P_dst = src_stage.partitions, dst_stage.partitions
        local_src = [q for q in range(P_src) if self.owner(q, si.src) == me]
        local_dst = [p for p in range(P_dst) if self.owner(p, dst_stage.id) == me]
        sends, ids = [], []
        for r in range(W):
            lst = []
            for q in local_src:
                v = self.channels[(si.src, q)]
                for p in range(P_dst):
                    if self.owner(p, dst_stage.id) == r:
                        lst.append(self._port_of(si, v, p))
            sends.append(lst)
        for r in range(W):
            ids.append([(q, p) for q in range(P_src) if self.owner(q, si.src) == r for p in local_dst])
        got = self._transport(dst_stage, si, sends, ids)
        out = {p: [None] * P_src for p in local_dst}
        for r in range(W):
            for (q, p), x in got[r].items():
                out[p][q] = x
        self._drop_consumed(si.src, dst_stage.id)
        return out

    def _drop_consumed(self, src_id, consumer_id):
        """The exchange delivered copies: free the producer's tables now (not at the end of the
        consumer stage) when nothing else reads them, so a shuffle holds send + receive only
        while it runs and receive + output afterwards."""
        st = self.plan.stages
        if st[src_id].is_output or any(f["x"] == src_id for f in self.fused.values()):
            return
        if any(src_id == i.src for t in st if t.id != consumer_id and t.id > src_id for i in t.inputs):
            return
        if sum(1 for i in st[consumer_id].inputs if i.src == src_id) > 1:
            return
        for key in [k for k in self.channels if k[0] == src_id]:
            del self.channels[key]

    # ------------------------------------------------------------------ vertex execution
    def _fault(self, s, p, version):
        for f in self.faults:
            if f.get("stage") not in (None, s.id, s.name) or f.get("partition") not in (None, p):
                continue
            if f.get("version") not in (None, version):
                continue
            return f.get("kind", "fail")
        return None

    def _merge_streams(self, si, streams):
        if not streams:
            return None
        if len(streams) == 1 and isinstance(streams[0], GS.StreamedPart):
            return streams[0]            # a part file a streamed producer already wrote
        if all(isinstance(x, DeviceTable) for x in streams):
            return DeviceTable.concat(streams)
        objs = [x if isinstance(x, list) else _to_objects(x) for x in streams]
        return [y for o in objs for y in o]

    def run_vertex(self, s, p, version, raw_inputs, inject=True, cancel=None):
        fault = self._fault(s, p, version) if inject else None
        if fault == "kill" and CK.gang_epoch() == 0:
            # a LOST rank process (not a simulated one): the launcher relaunches the gang, which
            # resumes from the persisted stage outputs (first start only, or it would die again)
            log.warning("injected kill of rank %d in %s[%d]", self.world.rank, s.name, p)
            import signal
            os.kill(os.getpid(), signal.SIGKILL)
        if fault == "fail":
            raise RuntimeError(f"injected vertex failure {s.name}[{p}] v{version}")
        if fault and fault.startswith("slow"):
            t = float(fault.split(":")[1]) if ":" in fault else 1.0
            if cancel is not None:
                cancel.wait(t)
            else:
                time.sleep(t)
        if fault == "read_error" and s.inputs:
            q = next(iter(self._sources(s.inputs[0], p)), None)
            if q is not None:
                raise ChannelReadError(self.edge_ids[(self.vids[s.inputs[0].src][q], self.vids[s.id][p], 0)],
                                       f"injected read error on the channel {s.inputs[0].src}[{q}] -> {s.id}[{p}]")
        vctx = GpuVertexContext(p, s.partitions, self.vids[s.id][p], version, s, self.dev, self.world, self)
        if s.id not in self.part_stream_plans:
            self.part_stream_plans[s.id] = ST.partition_plan(self, s)
        if self.part_stream_plans[s.id] is not None:
            # read -> record-wise ops -> HashPartition -> ToStore(partfile) on one rank: every chunk's
            # ports appended to the output partitions' part files (runtime/streaming.py)
            try:
                with TRC.range(f"vertex {s.id}:{s.name}[{p}] v{version} (streamed partition)"):
                    return ST.run_partitioned(self, s, p, version, vctx, self.part_stream_plans[s.id])
            except ST.NotStreamable as e:
                log.info("%s: streamed partitioning declined (%s)", s.name, e)
                self.part_stream_plans[s.id] = None
        if s.id not in self.agg_plans:
            self.agg_plans[s.id] = SA.plan(self, s)
        if self.agg_plans[s.id] is not None:
            # read -> ... -> GroupBy / Distinct over a partition past the HBM budget: chunks folded
            # into hash-bucketed running states, spilled to pinned host memory when they outgrow it
            with TRC.range(f"vertex {s.id}:{s.name}[{p}] v{version} (streamed aggregation)"):
                out = SA.run(self, s, p, version, vctx, self.agg_plans[s.id])
            if fault == "crash":
                raise VertexCrash(f"injected crash of {s.name}[{p}] v{version} (output discarded)")
            return out
        if s.id not in self.stream_plans:
            self.stream_plans[s.id] = ST.streamable(self, s)
        if self.stream_plans[s.id] is not None:
            # read -> record-wise ops -> write, chunk by chunk in bounded HBM (runtime/streaming.py)
            try:
                with TRC.range(f"vertex {s.id}:{s.name}[{p}] v{version} (streamed)"):
                    out = ST.run(self, s, p, version, vctx, self.stream_plans[s.id], cancel)
            except ST.NotStreamable as e:
                log.info("%s: streamed execution declined (%s)", s.name, e)
                self.stream_plans[s.id] = None
                return self.run_vertex(s, p, version, raw_inputs, inject=False, cancel=cancel)
            if fault == "crash":
                os.remove(out.path)
                raise VertexCrash(f"injected crash of {s.name}[{p}] v{version} (output discarded)")
            return out
        inputs = [self._merge_streams(si, streams) for si, streams in zip(s.inputs, raw_inputs)]
        if len(s.ops) == 1 and s.ops[0]["op"] == "output" and len(inputs) == 1 and isinstance(inputs[0], GS.StreamedPart):
            return inputs[0]             # the output stage of a streamed partitioning: committed by rename
        data = None
        with TRC.range(f"vertex {s.id}:{s.name}[{p}] v{version}"):
            for i, op in enumerate(s.ops):
                if cancel is not None and cancel.is_set():
                    raise VertexCancelled(f"{s.name}[{p}] v{version}")
                args = inputs if i == 0 else [data]
                with TRC.range(op["op"]):
                    data = self._run_op(op, args, vctx, s)
        if fault == "crash":        # the attempt dies after doing its work: its output must not be used
            raise VertexCrash(f"injected crash of {s.name}[{p}] v{version} (output discarded)")
        return data

    def _run_op(self, op, args, vctx, s):
        name = op["op"]
        fn = G.OPS.get(name) if self.gpu_ok else None
        device_apply = name == "apply" and is_device_function(op["fn"])
        if fn is not None and (device_apply or all(a is None or isinstance(a, DeviceTable) for a in args)):
            try:
                out = fn(op, [a for a in args] if args else [], vctx)
                self.op_counts[(name, "device")] += 1
                return out
            except NotTraceable as e:
                self._fallback(s, name, str(e), args)
        elif fn is None or not self.gpu_ok:
            self._fallback(s, name, "host op" if fn is None or not self.gpu_ok else "host records in", args)
        objs = [(_to_objects(a) if not isinstance(a, list) else a) if a is not None else [] for a in args]
        out = V.OPS[name](op, objs, vctx)
        self.op_counts[(name, "host" if any(_records(a) for a in args) else "host-empty")] += 1
        return self._maybe_device(out, s, name)

    def _fallback(self, s, name, why, args):
        """Record a host fallback; refuse one that would pull more than HostFallbackMaxBytes of
        device data into Python objects (a silent cliff on a 100 GB partition) unless the context
        allows it (AllowHostFallback).  An operator over empty inputs only (no record to process,
        e.g. a partition a shuffle left empty, whose output type a kernel cannot infer) is noted
        apart: it moves no data."""
        nb = sum(_device_bytes(a) for a in args)
        if all(_records(a) == 0 for a in args):
            self.empty_host_ops.append((s.name, name, why))
            return
        self.fallbacks.append((s.name, name, why))
        props = self.ctx._props
        if self.gpu_ok and nb > int(props.get("HostFallbackMaxBytes") or 0) and not props.get("AllowHostFallback"):
            e = DryadLinqException(
                ErrorCode.OperatorNotSupported,
                f"{s.name}: operator {name} cannot run on the device ({why}) and its host fallback would move "
                f"{nb / 1e6:.1f} MB of HBM data into Python objects (> HostFallbackMaxBytes); set "
                f"AllowHostFallback=True to run it on the host anyway")
            e.retriable = False
            raise e

    def _maybe_device(self, out, s, opname):
        """Host op result -> device table when the records are columnar (keeps later ops on GPU)."""
        if not self.gpu_ok or not isinstance(out, list) or not out:
            return out
        if isinstance(out[0], list):           # multi-port host output
            return out
        try:
            t = from_objects(out, None, self.dev)
        except Exception:  # noqa: BLE001
            t = None
        return t if t is not None else out

    # ------------------------------------------------------------------ gang relaunch / resume
    def _persist_stage(self, s):
        """Copy this rank's outputs of a completed stage to the checkpoint store (persist policy
        of a job run under a relaunching launcher, runtime/checkpoint.py): written by the native
        part writer, timed per stage (a ``stage_persisted`` job event), skipped when it would pass
        the store's budget (``persist_skipped``) and dropped when it fails (``persist_failed``):
        persistence only saves work after a relaunch, it never fails a job."""
        me = self.world.rank
        t0 = time.time()
        mine = [p for p in range(s.partitions) if self.owner(p, s.id) == me and (s.id, p) in self.channels]
        if self.gpu_ok:
            torch.cuda.synchronize(self.dev)          # the stage's kernels are not part of the cost
        t0 = time.time()
        need = sum(CK.StageCheckpoint.nbytes(self.channels[(s.id, p)]) for p in mine)
        ev = dict(stage=s.name, rank=me, bytes=need, budget=self.ckpt.budget, used=self.ckpt.used)
        if self.ckpt.used + need > self.ckpt.budget:
            self.persist_stats[s.name] = dict(skipped="budget", bytes=need)
            self.g.event(json.dumps(dict(ev, ev="persist_skipped", reason="checkpoint budget")))
            log.warning("stage %s not persisted: %d bytes past the checkpoint budget (%d of %d used)",
                        s.name, need, self.ckpt.used, self.ckpt.budget)
            return
        saved = 0
        try:
            for p in mine:
                saved += self.ckpt.save(s.id, p, self.channels[(s.id, p)])
        except Exception as e:  # noqa: BLE001 (a resume aid: the stage simply reruns after a relaunch)
            for p in mine:
                self.ckpt.drop(s.id, p)
            self.persist_stats[s.name] = dict(failed=f"{type(e).__name__}: {e}")
            self.g.event(json.dumps(dict(ev, ev="persist_failed", error=f"{type(e).__name__}: {e}")))
            log.warning("stage %s not persisted: %s", s.name, e)
            return
        dt = time.time() - t0
        self.persist_seconds += dt
        self.persist_stats[s.name] = dict(bytes=saved, ms=round(dt * 1e3, 2),
                                          GBps=round(saved / 1e9 / max(dt, 1e-9), 2), dir=self.ckpt.dir)
        self.g.event(json.dumps(dict(ev, ev="stage_persisted", bytes=saved, ms=round(dt * 1e3, 2))))

    def _resume_stage(self, s, ready, refresh, now) -> bool:
        """A relaunched gang: when EVERY rank holds the persisted outputs of all its partitions of
        stage s (one vote), load them instead of running the stage again."""
        me = self.world.rank
        mine = [p for p in range(s.partitions) if self.owner(p, s.id) == me]
        have = all(self.ckpt.has(s.id, p) for p in mine)
        from ..parallel import shuffle as SH
        if not all(ok for ok, _ in SH.gang_status(have, 0, self.world)):
            return False
        dev = self.dev if self.gpu_ok else torch.device("cpu")
        for p in mine:
            self.channels[(s.id, p)] = self.ckpt.load(s.id, p, dev)
        refresh()
        for p in range(s.partitions):
            vid = self.vids[s.id][p]
            ver = ready.pop(vid)
            self.g.on_running(vid, ver, self.owner(p, s.id), now())
            self.g.on_completed(vid, ver, now(), 0, 0)
        self.recovery.append(("resumed", s.name))
        self.g.event(json.dumps({"ev": "stage_resumed", "t": now(), "stage": s.name, "partitions": s.partitions,
                                 "epoch": CK.gang_epoch()}))
        return True

    # ------------------------------------------------------------------ main loop
    def run(self):
        g = self.g
        W, me = self.world.size, self.world.rank
        t_start = time.time()
        now = lambda: time.time() - t_start  # noqa: E731
        g.start(now())
        if self.ckpt is not None and CK.gang_epoch() == 0:
            # a first start never resumes: drop what an earlier run left under this job's key
            for st in self.plan.stages:
                for p in range(st.partitions):
                    if self.owner(p, st.id) == me:
                        self.ckpt.drop(st.id, p)
        if CK.gang_epoch() > 0:
            g.event(json.dumps({"ev": "gang_relaunch", "t": now(), "epoch": CK.gang_epoch(),
                                "reason": os.environ.get("DRYAD_GANG_RELAUNCH_REASON", ""),
                                "checkpoint": self.ckpt.dir if self.ckpt is not None else None}))
        ready = {}

        def refresh():
            for it in g.take_ready(1 << 30, now()):
                ready[it.vertex] = it.version

        self.place = self._placement()
        self.fused = self._find_fused_orderby()
        self.external = self._plan_external()
        for sid, e in self.external.items():
            self.fused.pop(sid, None)
            self.skipped.update(e["skip"])
        for sid in list(self.external) + list(self.fused):
            if self.plan.stages[sid].partitions > 1 and sid not in self.gang_stages:
                self.g.set_gang(self.vids[sid])      # one collective program: its vertices restart together
                self.gang_stages.add(sid)
        self.lazy_gen_stages = self._lazy_gen_reads()
        self.pitch_gen_stages = self._pitch_gen_reads()
        fused_first = {f["stages"][0]: mid for mid, f in self.fused.items()}
        active_fused = {}
        self.fused_joins = FJ.find(self.plan) if self.gpu_ok else {}
        self.grace_joins = GS.find(self.plan) if self.gpu_ok else {}
        join_first = {min(d["stages"]): jid for jid, d in list(self.fused_joins.items()) + list(self.grace_joins.items())}
        self.stream_shuffles = SSH.find(self.plan) if self.gpu_ok else {}
        shuffle_first = {d["a"]: bid for bid, d in self.stream_shuffles.items()}
        precomputed = {}
        stage_events = []          # (timing key, host seconds, start event, end event)
        t_stages = time.time()
        self.phases["setup"] = t_stages - t_start
        for s in self.plan.stages:
            t0 = time.time()
            ev0 = None
            if self.gpu_ok:
                ev0 = torch.cuda.Event(enable_timing=True)
                ev0.record(torch.cuda.current_stream(self.dev))
            status, err = 0, ""
            if s.id in join_first:
                jid = join_first[s.id]
                out, rest, how = None, [], ""
                if jid in self.fused_joins:
                    out, rest, how = self._try_fused_join(self.fused_joins[jid]), self.fused_joins[jid]["rest"], \
                        "fused grace join"
                if out is None and jid in self.grace_joins:
                    desc = self.grace_joins[jid]
                    lay = GS.vote(desc, self)
                    if lay is not None:
                        out, rest, how = self._attempt_stage(self.plan.stages[jid], lambda: GS.run(desc, self, lay)), \
                            [], "grace join stage"
                if out is not None:
                    precomputed[jid] = (out, rest)
                    body = (lambda d=self.fused_joins[jid]: FJ.run(d, self, FJ.vote(d, self))) \
                        if how == "fused grace join" else (lambda d=desc, ly=lay: GS.run(d, self, ly))
                    self.precomputed_bodies[jid] = (body, rest)
                    self.skipped.update((self.fused_joins.get(jid) or self.grace_joins[jid])["stages"])
                    self.timings[f"{jid}:Join({how})"] = time.time() - t0
            if s.id in shuffle_first:
                bid = shuffle_first[s.id]
                desc = self.stream_shuffles[bid]
                lay = SSH.vote(desc, self)
                if lay is not None:
                    body = (lambda d=desc, ly=lay: SSH.run(d, self, ly))
                    out = self._attempt_stage(self.plan.stages[bid], body)
                    if out is not None:
                        precomputed[bid] = (out, [])
                        self.precomputed_bodies[bid] = (body, [])
                        self.skipped.update(desc["stages"])
                        self.timings[f"{bid}:{self.plan.stages[bid].name}(streamed shuffle)"] = time.time() - t0
            if s.id in precomputed:
                refresh()
                outs, rest = precomputed.pop(s.id)
                for p, v in outs.items():
                    vctx = GpuVertexContext(p, s.partitions, self.vids[s.id][p], 0, s, self.dev, self.world, self)
                    for op in rest:                 # the join stage's program after the aggregate
                        v = self._run_op(op, [v], vctx, s)
                    self.channels[(s.id, p)] = v
                for p in range(s.partitions):
                    vid = self.vids[s.id][p]
                    ver = ready.pop(vid)
                    g.on_running(vid, ver, self.owner(p, s.id), now())
                    g.on_completed(vid, ver, now(), 0, 0)
                self._release(s)
                continue
            if s.id in fused_first:
                mid = fused_first[s.id]
                if self._fused_applicable(self.fused[mid]):
                    active_fused[mid] = self.fused[mid]
                    self.skipped.update(self.fused[mid]["stages"])
                else:
                    self._materialize(self.fused[mid]["x"])
            if s.id in self.skipped:
                refresh()
                for p in range(s.partitions):
                    vid = self.vids[s.id][p]
                    ver = ready.pop(vid)
                    g.on_running(vid, ver, self.owner(p, s.id), now())
                    g.on_completed(vid, ver, now(), 0, 0)
                self.timings[f"{s.id}:{s.name}(fused)"] = 0.0
                continue
            if s.id in self.external:
                e = self.external[s.id]
                out = self._run_gang(s, lambda: self._run_external(s, e), ready, refresh, now)
                self.channels[(s.id, me)] = out
                self._release(s)
                self.timings[f"{s.id}:{s.name}(out-of-core OrderBy)"] = time.time() - t0
                continue
            if s.id in active_fused:
                f = active_fused[s.id]
                out = self._run_gang(s, lambda: self._run_fused(s, f), ready, refresh, now,
                                     restore=lambda reread: self._restore_fused_input(f, reread))
                self.channels[(s.id, me)] = out
                self._release(s)
                if self.gpu_ok:
                    torch.cuda.synchronize(self.dev)
                self.timings[f"{s.id}:{s.name}(fused OrderBy)"] = time.time() - t0
                continue
            if self.ckpt is not None and self._resume_stage(s, ready, refresh, now):
                self._release(s)
                self.timings[f"{s.id}:{s.name}(resumed)"] = time.time() - t0
                continue
            if self.world.size > 1 and self._speculate(s):
                self._run_stage_speculative(s, ready, refresh, now)
            else:
                self._run_stage(s, ready, refresh, now)
            if self.ckpt is not None:
                self._persist_stage(s)
            self._release(s)
            # no synchronize between stages: the next stage's launches queue behind this one's
            # (a k-means iteration's four stages left the GPU idle while the host set up the
            # next); the stage time is its GPU span (events) or its host time, if longer
            if ev0 is not None:
                ev1 = torch.cuda.Event(enable_timing=True)
                ev1.record(torch.cuda.current_stream(self.dev))
                stage_events.append((f"{s.id}:{s.name}", time.time() - t0, ev0, ev1))
            else:
                self.timings[f"{s.id}:{s.name}"] = time.time() - t0
        if stage_events:
            stage_events[-1][3].synchronize()
            for key, host_s, ev0, ev1 in stage_events:
                self.timings[key] = max(host_s, ev0.elapsed_time(ev1) / 1e3)
        t_commit = time.time()
        self.phases["stages"] = t_commit - t_stages
        committed = self._commit()
        if self.pool is not None:
            for b in set(self.row_sets.values()):
                self.pool.release(b)
        self.phases["commit"] = time.time() - t_commit
        return dict(committed=committed, fallbacks=self.fallbacks, timings=self.timings, transports=self.transports,
                    op_counts={f"{k[0]}:{k[1]}": v for k, v in self.op_counts.items()},
                    empty_host_ops=self.empty_host_ops,
                    placement=self.place, moved={f"{k[0]}:{k[1]}": v for k, v in self.moved.items()},
                    write=dict(bytes=self.write_stats.bytes, seconds=round(self.write_stats.seconds, 4),
                               recycled_parts=self.recycled_parts),
                    phases={k: round(v, 4) for k, v in self.phases.items()},
                    read=dict(bytes=self.read_stats.bytes, seconds=round(self.read_stats.seconds, 4)),
                    sort_path=getattr(self, "last_sort_path", None),
                    exchange=(self.last_sort_stats.exchange_report() if getattr(self, "last_sort_stats", None)
                              is not None and self.last_sort_stats.rounds > 1 else None),
                    streamed={f"{k[0]}:{k[1]}": v for k, v in self.stream_stats.items()},
                    statistics=json.loads(g.statistics_json()), events=[json.loads(e) for e in g.drain_events()],
                    external_sort=getattr(self, "extsort_stats", None), join=getattr(self, "join_stats", None),
                    recovery=self.recovery, persist_seconds=round(self.persist_seconds, 4),
                    persist=dict(self.persist_stats))

    # ------------------------------------------------------------------ fault-tolerant stage execution
    def _run_stage(self, s, ready, refresh, now):
        """Run every vertex of stage s to completion, SPMD.  Rounds: each rank runs one attempt of
        each of its ready vertices, the attempt reports are all-gathered and every rank replays all
        of them, in rank order, on its JobGraph, so the version state machine (DrVertex.cpp:1042-1171,
        DrGraph.cpp:392-456) reaches identical decisions everywhere without further messages:

          * a failed attempt is re-executed from the same delivered inputs (HBM-resident), up to
            MaxVertexFailures, then the job aborts on every rank;
          * a failure inside a gang stage (a collective exchange's consumers) restarts every member;
          * a read error blames the producing vertex: its completed version is invalidated and it
            is re-executed on its owner (its own inputs re-delivered, released channels rebuilt from
            lineage), then the channel is delivered again.
        """
        g, W, me = self.g, self.world.size, self.world.rank
        local = [p for p in range(s.partitions) if self.owner(p, s.id) == me]
        raw, need_gather = None, True
        while True:
            if need_gather:
                raw = self._gather_inputs(s, recover=raw is not None)
                need_gather = False
            refresh()
            results, report = {}, []
            for p in local:
                vid = self.vids[s.id][p]
                if g.completed_version(vid) >= 0 or vid not in ready:
                    continue
                ver = ready[vid]
                try:
                    results[vid] = self.run_vertex(s, p, ver, raw[p])
                    report.append((vid, ver, "ok", -1, "", True))
                except ChannelReadError as e:
                    report.append((vid, ver, "read_error", e.edge, str(e), True))
                    self._dump_restart(s, p, ver, raw[p], str(e))
                except Exception as e:  # noqa: BLE001
                    self._last_exc = e
                    report.append((vid, ver, "fail", -1, f"{type(e).__name__}: {e}",
                                   getattr(e, "retriable", True) is not False))
                    self._dump_restart(s, p, ver, raw[p], f"{type(e).__name__}: {e}")
            reports = [report]
            if W > 1:
                # common case (every attempt succeeded): one small tensor all-gather; every rank
                # rebuilds the others' reports from the replicated ready set.  Only a failure
                # somewhere pays for the pickled reports with their messages.
                bad = self._gather_if_any(report if any(x[2] != "ok" for x in report) else None)
                if bad is None:
                    reports = [[(self.vids[s.id][p], ready[self.vids[s.id][p]], "ok", -1, "", True)
                                for p in range(s.partitions) if self.owner(p, s.id) == r
                                and g.completed_version(self.vids[s.id][p]) < 0 and self.vids[s.id][p] in ready]
                               for r in range(W)]
                    assert reports[me] == report, (reports[me], report)
                else:
                    reports = self._gather_objects(report)
            fatal, blamed = None, []
            for r in range(W):
                for vid, ver, kind, edge, err, retriable in reports[r]:
                    ready.pop(vid, None)
                    g.on_running(vid, ver, r, now())
                    if kind == "ok":
                        accepted, _ = g.on_completed(vid, ver, now(), 0, 0)
                        if accepted and r == me:
                            out = results[vid]
                            self.channels[(s.id, self.part_of[vid])] = out if out is not None else []
                        continue
                    if not retriable and fatal is None:
                        fatal = (r, err)
                    o = g.on_failed(vid, ver, now(), edge, err)
                    if o.action == 1:
                        blamed.append(o.invalidated_vertex)
                        self.recovery.append(("upstream", s.name, self.part_of[vid], o.invalidated_vertex))
                    elif s.id in self.gang_stages:
                        self.recovery.append(("gang_restart", s.name, self.part_of[vid]))
                    else:
                        self.recovery.append(("retry", s.name, self.part_of[vid]))
                    log.warning("vertex %s[%d] v%d failed (%s): %s", s.name, self.part_of[vid], ver, kind, err)
            if fatal is not None:
                if fatal[0] == me:
                    raise self._last_exc
                raise DryadLinqJobException(ErrorCode.JobToCreateTableFailed,
                                            f"job aborted: a vertex of stage {s.name} failed on rank {fatal[0]}: "
                                            f"{fatal[1]}")
            if g.failed():
                raise DryadLinqJobException(ErrorCode.JobToCreateTableFailed, g.failure(),
                                            inner=getattr(self, "_last_exc", None))
            for pv in sorted(set(blamed)):
                self._reexecute(pv, ready, refresh, now)
                need_gather = True
            if all(g.completed_version(v) >= 0 for v in self.vids[s.id]):
                return

    def _speculate(self, s) -> bool:
        """Duplicates only where a vertex's output may live on any rank: a leaf stage outside
        gangs whose consumers all fetch their inputs through owner() (the fused OrderBy / join /
        grace / out-of-core stages and the lazy or pitched reads feeding them assume partition p
        on its home rank, so they and their inputs are excluded)."""
        if not self.g_speculative or not self._duplicable(s, self.plan) or s.id in self.gang_stages:
            return False
        # (a gang consumer is fine: its exchange gathers every source partition from owner())
        special = set(self.skipped) | set(getattr(self, "lazy_gen_stages", ())) \
            | set(getattr(self, "pitch_gen_stages", ()))
        if self.gpu_ok:                  # (the fused OrderBy only runs on GPU ranks)
            for f in self.fused.values():
                special |= {f["x"], *f["stages"]}
        for d in (*self.fused_joins.values(), *self.grace_joins.values()):
            special |= set(d["stages"])
        for e in self.external.values():
            special |= set(e.get("skip", ()))
        return s.id not in special and not any(c in special for c in self.plan.consumers(s.id))

    def _run_stage_speculative(self, s, ready, refresh, now):
        """A leaf stage with speculative duplication (DrManagerBase::CheckForDuplicates,
        DrDefaultManager.cpp:664-714; outlier threshold DrStageStatistics.cpp:93-111).  Each rank runs
        its vertices on a worker thread; every SPEC_POLL seconds the ranks all-gather what started
        and finished and replay it on their JobGraphs in rank order (identical decisions everywhere,
        the latest rank clock as the common time).  A vertex running past the stage's outlier
        threshold gets a duplicate version on an idle rank (it re-reads its source); the first
        completion wins, its output stays on the winner's rank (``moved``) and later stages fetch
        it from there.  The losing attempt is cancelled at its next operator boundary (the
        reference kills the losing process), so every rank's worker drains before the stage ends
        and nothing runs on the device behind the next stage's collectives."""
        g, W, me = self.g, self.world.size, self.world.rank
        jobs, done = queue.Queue(), queue.Queue()
        dev = self.dev
        cancels = {}                                       # (p, version) -> Event of my live attempts

        def worker():
            if dev.type == "cuda":
                torch.cuda.set_device(dev)
            while True:
                item = jobs.get()
                if item is None:
                    return
                p, ver, dup = item
                try:
                    out = self.run_vertex(s, p, ver, [[] for _ in s.inputs], cancel=cancels[(p, ver)])
                    if dev.type == "cuda":
                        torch.cuda.synchronize(dev)
                    done.put((p, ver, dup, "ok", out, ""))
                except VertexCancelled:
                    self._drop_attempt(s, p, ver)
                    done.put((p, ver, dup, "cancelled", None, ""))
                except Exception as e:  # noqa: BLE001
                    done.put((p, ver, dup, "fail", None, f"{type(e).__name__}: {e}"))

        th = threading.Thread(target=worker, daemon=True, name=f"dryad-vertex-{s.id}")
        th.start()
        pending, started, outs = 0, [], {}

        def launch(p, ver, dup):
            nonlocal pending
            cancels[(p, ver)] = threading.Event()
            jobs.put((p, ver, dup))
            started.append((self.vids[s.id][p], ver, dup))
            pending += 1

        def take_ready():
            refresh()
            for p in range(s.partitions):
                vid = self.vids[s.id][p]
                if vid in ready:
                    ver = ready.pop(vid)
                    if g.completed_version(vid) < 0 and self.owner(p, s.id) == me:
                        launch(p, ver, False)
        try:
            take_ready()
            while True:
                finished, got = [], []
                try:                                           # wake at a local completion or a poll tick
                    got.append(done.get(timeout=self.SPEC_POLL))
                except queue.Empty:
                    pass
                while not done.empty():
                    got.append(done.get())
                for p, ver, dup, kind, out, err in got:
                    pending -= 1
                    cancels.pop((p, ver), None)
                    finished.append((self.vids[s.id][p], ver, dup, kind, err))
                    if kind == "ok":
                        outs[(p, ver)] = out
                rep = dict(t=now(), started=started, finished=finished, idle=pending == 0)
                started = []
                reps = [rep]
                if W > 1:
                    reps = shuffle.gather_json(rep, self.world)
                T = max(r["t"] for r in reps)
                for r, x in enumerate(reps):
                    for vid, ver, dup in x["started"]:
                        g.on_running(vid, ver, r, T)
                for r, x in enumerate(reps):
                    for vid, ver, dup, kind, err in x["finished"]:
                        p = self.part_of[vid]
                        if kind == "cancelled":
                            g.on_cancelled(vid, ver, T)
                        elif kind == "ok":
                            accepted, losers = g.on_completed(vid, ver, T, 0, 0)
                            if r == me:
                                out = outs.pop((p, ver))
                                if accepted:
                                    self.channels[(s.id, p)] = out if out is not None else []
                                elif (s.id, p) not in self.channels:
                                    self._drop_attempt(s, p, ver)     # a losing completion: free its HBM
                            if accepted:
                                if r != self.owner(p, s.id):
                                    self.moved[(s.id, p)] = r
                                if dup:
                                    self.recovery.append(("duplicate_won", s.name, p, r))
                                for lv, lver in losers:        # stop the losing attempt where it runs
                                    ev = cancels.get((self.part_of[lv], lver))
                                    if ev is not None:
                                        ev.set()
                        else:
                            g.on_failed(vid, ver, T, -1, err)
                            if g.completed_version(vid) < 0:
                                self.recovery.append(("retry", s.name, p))
                            log.warning("vertex %s[%d] v%d failed: %s", s.name, p, ver, err)
                if g.failed():
                    raise DryadLinqJobException(ErrorCode.JobToCreateTableFailed, g.failure())
                if all(g.completed_version(v) >= 0 for v in self.vids[s.id]) and \
                        not any(x["started"] for x in reps) and all(x["idle"] for x in reps):
                    return
                take_ready()                                   # retries of failed attempts
                idle = [r for r, x in enumerate(reps) if x["idle"]]
                if not idle:
                    continue
                dups = g.check_duplicates(T)
                refresh()                                      # the duplicates are placed here, not by owner
                for it in dups:
                    if ready.get(it.vertex) == it.version:
                        ready.pop(it.vertex)
                    p = self.part_of[it.vertex]
                    cand = [r for r in idle if r != self.owner(p, s.id)]
                    if not cand:
                        g.on_cancelled(it.vertex, it.version, T)
                        continue
                    r = cand[0]
                    idle.remove(r)
                    self.recovery.append(("duplicate", s.name, p, r))
                    log.info("duplicate of %s[%d] v%d on rank %d", s.name, p, it.version, r)
                    if r == me:
                        launch(p, it.version, True)
        finally:
            for ev in cancels.values():
                ev.set()
            jobs.put(None)
            th.join()

    SPEC_POLL = 0.02

    def _drop_attempt(self, s, p, ver):
        """A speculative attempt (s, p, ver) that lost or was cancelled on this rank: its pooled
        rows go back to the pool and its streamed part file (``<tmp part>.stream``) is removed."""
        bs = self.row_sets.get((s.id, p))
        if bs is not None and (s.id, p) not in self.channels and self.pool is not None:
            self.row_sets.pop((s.id, p), None)
            self.pool.release(bs)
        if s.is_output and getattr(s, "output", None):
            try:
                scheme, path, _ = parse_uri(s.output["uri"])
            except Exception:  # noqa: BLE001
                return
            if scheme in ("partfile", "file"):
                from ..io import partfile as PF
                f = PF.tmp_part_path(PF.default_base(path), p, self.vids[s.id][p], 0, ver) + ".stream"
                try:
                    os.remove(f)
                except OSError:
                    pass

    def _dump_restart(self, s, p, ver, streams, error):
        """Restart record of a failed GPU vertex attempt (DumpRestartCommand, dvertexpncontrol.cpp:
        348-736): its delivered inputs persisted under ``log/rerun/vertex-V.v/`` (device tables as
        tensor files + JSON layout, host records pickled) with the plan, so
        ``python -m dryad_amd.tools.replay`` re-runs this one vertex standalone.  Skipped past
        ``RerunInputsMaxBytes`` (default 1 GiB) of input."""
        jd = getattr(self, "job_dir", None)
        if not jd and getattr(self, "job_dir_factory", None) is not None:
            jd = self.job_dir = self.job_dir_factory()
        if not jd:
            return
        try:
            from ..tools import replay as RP
            nb = sum(_device_bytes(x) for inp in streams for x in inp)
            limit = int(self.ctx._props.get("RerunInputsMaxBytes") or (1 << 30))
            RP.dump(jd, self.plan, s, p, self.vids[s.id][p], ver, streams if nb <= limit else None, error)
        except Exception as e:  # noqa: BLE001 (a diagnostic aid must never fail the job)
            log.warning("could not write the restart record of %s[%d]: %s", s.name, p, e)

    def _reexecute(self, vid, ready, refresh, now):
        """Collective: re-run one invalidated producer vertex on its owner (DrVertex.cpp:1135-1158),
        its inputs delivered again (and rebuilt from lineage where they were released)."""
        st, p = self.plan.stages[self.stage_of[vid]], self.part_of[vid]
        me = self.world.rank
        if st.id in self.precomputed_bodies:
            # a fused stage's partitions come from one computation (its own key routing), so one
            # of them is rebuilt by running the whole fused stage again (every rank takes part)
            body, rest = self.precomputed_bodies[st.id]
            refresh()
            ver = ready.pop(vid)
            self.g.on_running(vid, ver, self.owner(p, st.id), now())
            outs = self._attempt_stage(st, body, first_version=ver)
            if outs is None:
                raise DryadLinqJobException(ErrorCode.JobToCreateTableFailed,
                                            f"re-execution of the fused stage {st.name} was declined")
            for q, v in outs.items():
                vctx = self._vertex_ctx(st, q, ver)
                for op in rest:
                    v = self._run_op(op, [v], vctx, st)
                self.channels[(st.id, q)] = v
            self.g.on_completed(vid, ver, now(), 0, 0)
            self.recovery.append(("rerun_fused", st.name, p))
            return
        raw = self._gather_inputs(st, only=[p], recover=True)
        refresh()
        ver = ready.pop(vid)
        self.g.on_running(vid, ver, self.owner(p, st.id), now())
        ok, err = True, ""
        if self.owner(p, st.id) == me:
            try:
                out = self.run_vertex(st, p, ver, raw[p])
                self.channels[(st.id, p)] = out if out is not None else []
            except Exception as e:  # noqa: BLE001
                ok, err = False, f"{type(e).__name__}: {e}"
        oks = [(ok, err)]
        if self.world.size > 1:
            oks = shuffle.gather_json([ok, err], self.world)
        bad = next((x for x in oks if not x[0]), None)
        if bad is not None:
            raise DryadLinqJobException(ErrorCode.JobToCreateTableFailed,
                                        f"re-execution of {st.name}[{p}] after a read error failed: {bad[1]}")
        self.g.on_completed(vid, ver, now(), 0, 0)

    def _rematerialize(self, sid):
        """Collective: rebuild a stage's released output channels from lineage (its inputs, rebuilt
        recursively) so an input can be delivered again after a read error.  A cache refill, not a
        new vertex version: no JobGraph attempt is recorded."""
        st = self.plan.stages[sid]
        raw = self._gather_inputs(st, recover=True)
        for p, streams in raw.items():
            self.channels[(sid, p)] = self.run_vertex(st, p, max(0, self.g.completed_version(self.vids[sid][p])),
                                                      streams, inject=False)
        self.recovery.append(("rematerialize", st.name))

    def _try_fused_join(self, desc):
        """Run a Join + aggregate idiom as one fused grace join stage (runtime/fused_join.py) when
        every rank can; None (the plan's stages run as compiled) otherwise."""
        lay = FJ.vote(desc, self)
        if lay is None:
            return None
        return self._attempt_stage(self.plan.stages[desc["join"]], lambda: FJ.run(desc, self, lay))

    def _attempt_stage(self, st, body, first_version: int = 0):
        """Versioned, voted attempts of a precomputed (fused) join stage, whose vertices the main
        loop completes later.  Attempts are voted like a gang stage's (``_run_gang``): injected
        faults on the stage's partitions are agreed before the body (fail, read_error) or after it
        (crash), and a failed attempt is re-run from its inputs (generated, HBM-resident or stored,
        so re-readable) until MaxVertexFailures.  An exception raised on EVERY rank (e.g. an
        allocation the budget check let through) means every rank left the body together: None,
        the compiled stages run instead.  One raised on some ranks only leaves the others in a
        collective; the communicator's error handling then ends the job (parallel/comm.py)."""
        me = self.world.rank
        mine = [p for p in range(st.partitions) if self.owner(p, st.id) == me]
        limit = int(getattr(self.ctx, "MaxVertexFailures", 6) or 6)
        outcome = None
        for version in range(first_version, first_version + limit):
            faults = {p: self._fault(st, p, version) for p in mine}
            pre = next(((p, k) for p, k in faults.items() if k in ("fail", "read_error")), None)
            outcome = self._vote(None if pre is None else (pre[0], pre[1], f"injected {pre[1]} of {st.name}[{pre[0]}]"))
            out = None
            real = False
            if outcome is None:
                err = None
                try:
                    out = body()
                    crash = next((p for p, k in faults.items() if k == "crash"), None)
                    if crash is not None:
                        err = (crash, "crash", f"injected crash of {st.name}[{crash}] (output discarded)")
                except Exception as e:  # noqa: BLE001
                    err = (mine[0] if mine else 0, "exception", f"{type(e).__name__}: {e}")
                    log.warning("%s attempt %d failed: %s", st.name, version, e)
                outcome = self._vote(err)
                real = outcome is not None and len(outcome) == self.world.size and \
                    all(e[1] == "exception" for _, e in outcome)
            if outcome is None:
                return out
            if real:
                self.recovery.append(("fused_stage_declined", st.name, outcome[0][1][2]))
                return None
            for _, (p, kind, _msg) in outcome:
                self.recovery.append(("upstream" if kind == "read_error" else "gang_restart", st.name, p))
        raise DryadLinqJobException(ErrorCode.JobToCreateTableFailed,
                                    f"{st.name} failed {limit} times: {outcome[0][1][2]}")

    def _vertex_ctx(self, s, p, version=0):
        return GpuVertexContext(p, s.partitions, self.vids[s.id][p], version, s, self.dev, self.world, self)

    def _release(self, s):
        later = {i.src for st in self.plan.stages if st.id > s.id for i in st.inputs}
        later |= {f["x"] for mid, f in self.fused.items() if mid > s.id}
        for (sid, p) in list(self.channels):
            if sid <= s.id and sid not in later and not self.plan.stages[sid].is_output:
                del self.channels[(sid, p)]

    # ------------------------------------------------------------------ outputs
    def _commit(self):
        W, me = self.world.size, self.world.rank
        committed = {}
        for s in self.plan.stages:
            if not s.is_output:
                continue
            uri = s.output["uri"]
            scheme, path, _ = parse_uri(uri)
            local = {p: self.channels[(s.id, p)] for p in range(s.partitions) if self.owner(p, s.id) == me}
            if scheme == "hbm":
                tabs = {p: (v if isinstance(v, DeviceTable) else v) for p, v in local.items()}
                pins = [self.row_sets[(s.id, p)] for p in local if (s.id, p) in self.row_sets]
                for b in pins:
                    self.pool.pin(b)
                provider_for(uri).put(uri, {"dtype": s.dtype, "partitions": s.partitions, "local": tabs,
                                            "owner_of": {p: self.owner(p, s.id) for p in range(s.partitions)},
                                            "bytes": sum(_object_bytes(v) for v in tabs.values()),
                                            "pins": pins, "pool": self.pool})
                committed[uri] = s.partitions
            elif scheme == "host":
                from ..io.hosttable import HostColumns
                tabs = {}
                for p, v in local.items():
                    if isinstance(v, (HostRows, HostColumns)):        # streamed into the host tier
                        tabs[p] = v
                    elif isinstance(v, DeviceTable) and v.rows is not None and v.device.type == "cuda":
                        tabs[p] = HostRows.from_tensor(v.rows, v.shape.key_off, v.shape.key_len)
                    elif isinstance(v, DeviceTable) and v.device.type == "cuda" and v.heap is None and not v.strs:
                        h = HostColumns(v.shape)            # columns DMA'd into pinned host memory
                        h.append(v)
                        tabs[p] = h
                    else:
                        tabs[p] = _to_objects(v) if not isinstance(v, list) else v
                provider_for(uri).put(uri, {"dtype": s.dtype, "partitions": s.partitions, "local": tabs,
                                            "owner_of": {p: self.owner(p, s.id) for p in range(s.partitions)}})
                committed[uri] = s.partitions
            elif scheme in ("partfile", "file") and self._commit_partfile(s, uri, path, local):
                committed[uri] = s.partitions
            else:
                # host stores: every rank ships its partitions' records to rank 0, which writes them
                objs = {p: _to_objects(v) if not isinstance(v, list) else v for p, v in local.items()}
                gathered = [None] * W
                if W > 1:
                    dist.all_gather_object(gathered, objs)
                else:
                    gathered = [objs]
                if me == 0:
                    parts = {}
                    for d in gathered:
                        parts.update(d)
                    ordered = [parts[p] for p in range(s.partitions)]
                    prov = provider_for(uri)
                    if prov.exists(uri):
                        if s.output.get("delete_if_exists") or s.output.get("temp"):
                            prov.delete(uri)
                        else:
                            raise DryadLinqException(ErrorCode.JobToCreateTableFailed, f"output {uri} exists")
                    from .. import types as T
                    dt = s.dtype
                    if dt is None or dt == T.Pickle:
                        flat = [x for part in ordered for x in part[:100]]
                        dt = T.infer_common_type(flat) if flat else T.Int32
                    prov.write_table(uri, ordered, dt)
                if W > 1:
                    self.world.barrier()
                committed[uri] = s.partitions
            qn = s.output.get("qnode")
            if qn is not None:
                qn.args["_executed"] = True
        return committed


def _commit_partfile_impl(runner, s, uri, path, local):
    """Partfile output written in parallel: every rank encodes its own partitions (device codec
    for fixed-width columnar tables, host encoder otherwise) into tmp part files, rank 0 commits
    the metadata by rename (reference DrPartitionFile.cpp:463-600).  Returns False when the
    record type has to be inferred from the data on the host (then rank 0 writes everything)."""
    from .. import types as T
    from ..io import binary as B
    from ..io import partfile as PF
    from ..io import writer as WR
    from ..ops import codec as CD
    from .jobmanager import write_schema
    W, me = runner.world.size, runner.world.rank
    dt = s.dtype
    rows_fmt = any(isinstance(v, HostRows) or (isinstance(v, DeviceTable) and v.rows is not None and
                                               v.shape.kind == "rows" and v.device.type == "cuda")
                   or (isinstance(v, GS.StreamedPart) and v.rows is not None)
                   for v in local.values())
    streamed = [v for v in local.values() if isinstance(v, GS.StreamedPart)]
    if streamed and (dt is None or dt == T.Pickle):
        dt = streamed[0].dtype
    if dt is None or dt == T.Pickle:
        # a plan that does not know the record type (e.g. a Select to tuples): the device tables'
        # columns define it, so the parts are device-encoded instead of going through host records
        for v in local.values():
            if isinstance(v, DeviceTable) and v.device.type == "cuda":
                got = GS._table_dtype(v)
                if got is not None:
                    dt = got
                    break
    if W > 1 and (s.dtype is None or s.dtype == T.Pickle):
        # every rank takes the record type the first rank that knows one learnt (ranks without
        # rows have none); the plan-level condition keeps every rank in this collective
        allts = shuffle.gather_json(None if dt is None or dt == T.Pickle else T.dtype_to_json(dt), runner.world)
        got = next((x for x in allts if x is not None), None)
        dt = T.dtype_from_json(got) if got is not None else dt
    if not rows_fmt and (dt is None or dt == T.Pickle):
        return False
    prov = provider_for(uri)
    if me == 0 and prov.exists(uri):
        if s.output.get("delete_if_exists") or s.output.get("temp"):
            try:                    # the old parts move aside now and are unlinked in the background
                prov.delete(uri, background=True)
            except TypeError:
                prov.delete(uri)
        else:
            raise DryadLinqException(ErrorCode.JobToCreateTableFailed, f"output {uri} exists")
    if W > 1:
        runner.world.barrier()
    base = PF.default_base(path)
    os.makedirs(os.path.dirname(base) or ".", exist_ok=True)
    mine = {}
    state = dict(fmt_extra=None, bounds={}, noted=0)

    def note_bounds(v=None, measured=None):
        """Union of the integer columns' [min, max] over this rank's written partitions (kept in
        the table's schema, so a later read knows them as a generator's columns do: a GroupBy or
        join packing by value width skips its min / max pass).  ``measured``: a streamed part's
        own union (its writer measured every chunk)."""
        from ..gpu.stats import BoundsAcc
        if measured is None:
            acc = BoundsAcc()
            acc.add(v)
            measured = acc.result()
        if measured is None:
            return
        state["noted"] += 1
        for f, (lo, hi) in measured.items():
            old = state["bounds"].get(f)
            state["bounds"][f] = [lo, hi] if old is None else [min(old[0], lo), max(old[1], hi)]

    def write_parts():
        for p, v in local.items():
            tmp = PF.tmp_part_path(base, p, runner.vids[s.id][p], 0, 0)
            if isinstance(v, GS.StreamedPart) and v.bounds is not None and v.rows is None:
                note_bounds(measured=v.bounds)
            if isinstance(v, GS.StreamedPart) and isinstance(v.path, list):    # split over part files
                mine[p] = []
                for j, f in enumerate(v.path):
                    os.replace(f, f"{tmp}.{j}")
                    if os.path.exists(f + PF.INDEX_SUFFIX):          # the piece's block index
                        os.replace(f + PF.INDEX_SUFFIX, f"{tmp}.{j}" + PF.INDEX_SUFFIX)
                    mine[p].append(f"{tmp}.{j}")
                continue
            if isinstance(v, GS.StreamedPart):          # written bucket / chunk by chunk by its stage
                os.replace(v.path, tmp)
                if os.path.exists(v.path + PF.INDEX_SUFFIX):         # the block index of string records
                    os.replace(v.path + PF.INDEX_SUFFIX, tmp + PF.INDEX_SUFFIX)
                if v.rows is not None:
                    state["fmt_extra"] = dict(v.rows)
                mine[p] = tmp
                continue
            if rows_fmt:
                # raw fixed-width rows: device rows or the pinned host tier (out-of-core sort output)
                if isinstance(v, DeviceTable):
                    mine[p] = _write_split(runner, tmp, v.rows[: v.n], v.n, v.rows.shape[1])
                    state["fmt_extra"] = dict(stride=v.rows.shape[1], key_off=v.shape.key_off, key_len=v.shape.key_len)
                    continue
                if getattr(v, "path", None) and os.path.exists(v.path):
                    # disk tier: the rows already are a file; flush it and rename it into place
                    v.flush()
                    if v.n * v.stride != os.path.getsize(v.path):
                        os.truncate(v.path, v.n * v.stride)
                    os.replace(v.path, tmp)
                else:
                    WR.write_device(tmp, v.rows[: v.n], stats=runner.write_stats)
                state["fmt_extra"] = dict(stride=v.stride, key_off=v.key_off, key_len=v.key_len)
                mine[p] = tmp
                continue
            data = CD.encode(v, dt) if isinstance(v, DeviceTable) and v.device.type == "cuda" else None
            index = None
            if data is None and isinstance(v, DeviceTable) and v.device.type == "cuda":
                enc = CD.encode_var(v, dt)              # strings: device encoder + block index
                if enc is not None:
                    data, boffs = enc
                    index = (v.n, data.numel(), boffs.cpu().numpy(), CD.BLOCK)
            if runner.ctx.OutputDataCompressionScheme.value != 0:
                import gzip
                raw = data.cpu().numpy().tobytes() if data is not None else \
                    B.encode_records(dt, _to_objects(v) if not isinstance(v, list) else v)
                with open(tmp, "wb") as f:
                    f.write(gzip.compress(raw, compresslevel=6))
            elif data is not None:
                # device-encoded records: HBM -> pinned ring -> native writer threads
                note_bounds(v)
                if index is None and v.n and data.numel() % v.n == 0:      # fixed-width records
                    mine[p] = _write_split(runner, tmp, data, v.n, data.numel() // v.n)
                    continue
                WR.write_device(tmp, data, stats=runner.write_stats)
                if index is not None:
                    PF.write_index(tmp, index[0], index[1], index[2], index[3])
            else:
                B.write_records(tmp, dt, _to_objects(v) if not isinstance(v, list) else v)
            mine[p] = tmp

    try:
        write_parts()
    except BaseException:
        # this rank's uncommitted part files (tmp, split pieces, block indexes) go with the failure
        prefixes = [PF.tmp_part_path(base, p, runner.vids[s.id][p], 0, 0) for p in local]
        d = os.path.dirname(base) or "."
        for fn in os.listdir(d):
            q = os.path.join(d, fn)
            if any(q.startswith(x) for x in prefixes):
                try:
                    os.remove(q)
                except OSError:
                    pass
        raise
    fmt_extra = state["fmt_extra"]
    empty = sum(1 for v in local.values() if (isinstance(v, DeviceTable) and v.n == 0) or (isinstance(v, list) and not v))
    # the bounds hold for the table only when every non-empty partition was measured
    bounds = state["bounds"] if state["noted"] + empty == len(local) else None
    gathered = [None] * W
    gathered_fmt = [None] * W
    if W > 1:
        # part-file paths, the rows format and the column bounds (JSON over one tensor all-gather)
        got = shuffle.gather_json([[[int(p), v] for p, v in mine.items()], fmt_extra, bounds], runner.world)
        gathered = [{p: v for p, v in x[0]} for x in got]
        gathered_fmt = [x[1] for x in got]
        allb = [x[2] for x in got]
    else:
        gathered = [mine]
        allb = [bounds]
    if me == 0:
        parts = {}
        for d in gathered:
            parts.update(d)
        chosen = []                 # a split partition contributes its part files in order
        for p in range(s.partitions):
            chosen.extend(parts[p] if isinstance(parts[p], list) else [parts[p]])
        PF.commit_parts(path, base, chosen)
        if rows_fmt:
            extras = [x for x in gathered_fmt if x] if W > 1 else [fmt_extra]
            write_schema(path, dt, "rows", **(extras[0] if extras and extras[0] else {}))
        else:
            extra = {}
            if all(b is not None for b in allb) and any(allb):
                union = {}
                for b in allb:
                    for f, (lo, hi) in b.items():
                        u = union.get(f)
                        union[f] = [lo, hi] if u is None else [min(u[0], lo), max(u[1], hi)]
                extra["bounds"] = union
            write_schema(path, dt, "binary", **extra)
    if W > 1:
        runner.world.barrier()
    if me == 0:
        PF.drop_recycled(base)          # every rank has claimed what it overwrote
    return True


def _write_split(runner, tmp: str, data, n: int, rec: int):
    """Write ``n`` fixed-width records of ``rec`` bytes (``data``) to the part file ``tmp``, or, with
    ``PartFileSplitBytes`` set and at least that many bytes, to several part files at once split at
    record boundaries (io/writer.write_device_pieces).  Returns the tmp path or the list of them."""
    from ..io import partfile as PF
    from ..io import writer as WR
    split = int(runner.ctx.PartFileSplitBytes or 0)
    nbytes = n * rec
    k = min(WR.SPLIT_MAX, nbytes // split) if split > 0 else 1
    if k <= 1:
        WR.write_device(tmp, data, stats=runner.write_stats)
        return tmp
    per = -(-n // k)
    bounds = [min(n, j * per) * rec for j in range(k + 1)]
    paths = [f"{tmp}.{j}" for j in range(k)]
    # parts of a table this job replaced are overwritten in place (io/partfile.py RECYCLE_DIR)
    got = PF.claim_recycled(paths)
    runner.recycled_parts += got
    WR.write_device_pieces(paths, data, bounds, stats=runner.write_stats, reuse=got > 0)
    return paths


GpuJobRunner._commit_partfile = lambda self, s, uri, path, local: _commit_partfile_impl(self, s, uri, path, local)


class _JobDirWriter:
    """Writes GPU job directories (plan / QueryPlan.xml / explain, events, statistics) on a daemon
    thread.  Serialising and writing them took ~0.6 ms of host time per job, in series with the
    device work of the next job (5% of a k-means iteration); queued, they run while the job thread
    waits on the GPU.  ``flush()`` (``GpuExecutor.last_job_dir``, the job browser, exit) waits
    for the queue."""

    def __init__(self):
        self.q: queue.Queue = queue.Queue()
        self.thread = None
        self.lock = threading.Lock()

    def submit(self, fn, *args):
        with self.lock:
            if self.thread is None or not self.thread.is_alive():
                self.thread = threading.Thread(target=self._loop, daemon=True, name="dryad-jobdir-writer")
                self.thread.start()
        self.q.put((fn, args))

    def _loop(self):
        while True:
            fn, args = self.q.get()
            try:
                fn(*args)
            except Exception as e:  # noqa: BLE001  (bookkeeping must not fail a job)
                log.warning("job directory write failed: %s", e)
            finally:
                self.q.task_done()

    def flush(self):
        if self.thread is not None:
            self.q.join()


_JOB_DIR_WRITER = _JobDirWriter()
atexit.register(_JOB_DIR_WRITER.flush)


def flush_job_dirs():
    _JOB_DIR_WRITER.flush()


def _write_plan_files(d, plan):
    os.makedirs(os.path.join(d, "log"), exist_ok=True)
    with open(os.path.join(d, "plan.json"), "w") as f:
        f.write(plan.dumps())
    with open(os.path.join(d, "QueryPlan.xml"), "w") as f:   # the reference job directory's plan
        f.write(plan.to_xml())
    with open(os.path.join(d, "QueryGraph.txt"), "w") as f:
        f.write(plan.explain())


def _write_events(d, evs):
    with open(os.path.join(d, "log", "events.jsonl"), "w") as f:
        f.write("".join(json.dumps(e) + "\n" for e in evs))


def _write_json(path, obj):
    with open(path, "w") as f:
        json.dump(obj, f, indent=1, default=str)


class GpuExecutor(_BaseExecutor):
    def __init__(self, ctx):
        self.ctx = ctx
        w = get_world()
        if w.size == 1 and int(os.environ.get("WORLD_SIZE", "1")) > 1:
            w = init_world(device=ctx._props.get("Device"))             # launched by torchrun
        elif w.size == 1 and w.device.type == "cpu" and torch.cuda.is_available() \
                and ctx._props.get("Device", "cuda") != "cpu":
            w = World(0, 1, 0, torch.device("cuda", torch.cuda.current_device()), None)
        self.world = w
        self.last_result = None
        # per job (the last 1000): host fallbacks and device / host operator counts
        self.job_log = collections.deque(maxlen=1000)
        from ..gpu.pool import HbmPool
        self.pool = HbmPool(w.device) if w.device.type == "cuda" else None

    def _enter_job_thread(self):
        """Jobs run on a thread of their own, and the HIP current device is per thread (a new one
        starts on device 0): bind it to this rank's GPU, or the library's launches on the default
        (null) stream and its device queries would go to GPU 0 on every rank."""
        if self.world.device.type == "cuda" and self.world.device.index is not None:
            torch.cuda.set_device(self.world.device)

    def run_job(self, outs, handle):
        dev = self.world.device
        if dev.type == "cuda" and dev.index is not None and torch.cuda.current_device() != dev.index:
            torch.cuda.set_device(dev)
        t_job = time.perf_counter()
        plan = compile_queries(self.ctx, outs)
        t_compiled = time.perf_counter()
        faults = self.ctx._props.get("FaultInjection") or []
        for st in plan.stages:      # CheckExistence(deleteIfExists) at submission
            if st.is_output and st.output["uri"].startswith(("hbm://", "host://")):
                prov = provider_for(st.output["uri"])
                if prov.exists(st.output["uri"]):
                    if st.output.get("delete_if_exists") or st.output.get("temp"):
                        prov.delete(st.output["uri"])
                    else:
                        raise DryadLinqException(ErrorCode.JobToCreateTableFailed,
                                                 f"output {st.output['uri']} already exists")
        runner = GpuJobRunner(self.ctx, plan, self.world, faults, self.pool)
        root = CK.from_env(self.ctx)
        if root is not None:
            GpuExecutor._ckpt_seq += 1
            budget = self.ctx._props.get("CheckpointBudgetBytes")
            runner.ckpt = CK.StageCheckpoint(root, CK.job_key(GpuExecutor._ckpt_seq, plan),
                                             budget=int(budget) if budget else None)
        job_dir = self._job_dir(plan) if self.world.rank == 0 else None
        runner.job_dir = job_dir
        self.last_job_dir = job_dir
        if self.ctx._props.get("KeepJobDirectories", True):
            runner.job_dir_factory = lambda: self._rank_job_dir(plan)    # restart records of rank > 0
        t0 = time.time()
        res = None
        from ..ops import tuning
        try:
            with tuning.scope(self.ctx):          # the job's operator strategies (context properties)
                res = runner.run()
        except BaseException as e:
            if job_dir:
                os.makedirs(os.path.join(job_dir, "log"), exist_ok=True)
                with open(os.path.join(job_dir, "log", "error.txt"), "w") as f:
                    f.write(str(e))
            raise
        finally:
            if job_dir:
                evs = res["events"] if res else [json.loads(e) for e in runner.g.drain_events()]
                _JOB_DIR_WRITER.submit(_write_events, job_dir, list(evs))
        if job_dir:
            st = dict(res.get("statistics") or {})
            st.update(executor="gpu", ranks=self.world.size, elapsed_s=time.time() - t0,
                      stage_seconds=res.get("timings"), host_fallbacks=res.get("fallbacks"),
                      transports=res.get("transports"), recovery=res.get("recovery"))
            _JOB_DIR_WRITER.submit(_write_json, os.path.join(job_dir, "statistics.json"), st)
        self.last_job_dir = job_dir
        t_sub = getattr(handle, "t_submit", None)
        res.setdefault("phases", {}).update(compile=round(t_compiled - t_job, 4),
                                            job=round(time.perf_counter() - t_job, 4),
                                            queued=None if t_sub is None else round(t_job - t_sub, 4))
        self.last_result = res
        self.job_log.append(dict(fallbacks=list(res["fallbacks"]), op_counts=dict(res["op_counts"])))
        self.last_plan = plan
        self.last_sort_path = getattr(runner, "last_sort_path", None)
        if handle is not None:
            handle.events.extend(res["events"])
        return res

    _seq = 0
    _ckpt_seq = 0              # jobs run by this process (the checkpoint key: same order after a relaunch)
    _last_job_dir = None

    @property
    def last_job_dir(self):
        """The last job's directory, with every file of it written (the writes are queued)."""
        _JOB_DIR_WRITER.flush()
        return self._last_job_dir

    @last_job_dir.setter
    def last_job_dir(self, d):
        self._last_job_dir = d

    def _job_dir(self, plan):
        """LocalJobs-style job directory (plan, explain, Calypso-style events, statistics) so
        ``python -m dryad_amd.tools.jobbrowser`` works on GPU jobs too."""
        if not self.ctx._props.get("KeepJobDirectories", True):
            return None
        from .executor import dryad_home
        GpuExecutor._seq += 1
        d = os.path.join(dryad_home(self.ctx), "LocalJobs", f"gpu-{os.getpid()}-{int(time.time() * 1000) % 10**9}-{GpuExecutor._seq}")
        _JOB_DIR_WRITER.submit(_write_plan_files, d, plan)      # creates the directory first
        return d

    def _rank_job_dir(self, plan):
        """Job directory of a non-zero rank (only for restart records of injected-fault runs)."""
        from .executor import dryad_home
        d = os.path.join(dryad_home(self.ctx), "LocalJobs",
                         f"gpu-rank{self.world.rank}-{os.getpid()}-{int(time.time() * 1000) % 10**9}")
        os.makedirs(os.path.join(d, "log"), exist_ok=True)
        return d

    def enumerate(self, q):
        node = q.node
        if node.op == "ToStore" and node.args.get("_executed"):
            uri = node.args["uri"]
            return self._read_back(uri, node.dtype)
        if node.op == "ToStore":
            self.ctx.SubmitAndWait(q)
            return self._read_back(node.args["uri"], node.dtype)
        from ..io.providers import unique_name
        tmp = "hbm://" + unique_name("enum")
        st = q.ToStore(tmp)
        st.node.args["_temp"] = True
        self.run_job([st], None)
        try:
            return self._read_back(tmp, st.node.dtype)
        finally:
            provider_for(tmp).delete(tmp)

    def _read_back(self, uri, dtype):
        if not uri.startswith(("hbm://", "host://")):
            return list(provider_for(uri).read_all(uri, dtype))
        ent = provider_for(uri).get(uri)
        mine = {p: _to_objects(v) if not isinstance(v, list) else v for p, v in ent["local"].items()}
        W = self.world.size
        if W > 1:
            gathered = [None] * W
            dist.all_gather_object(gathered, mine)
            allp = {}
            for d in gathered:
                allp.update(d)
        else:
            allp = mine
        return [x for p in range(ent["partitions"]) for x in allp.get(p, [])]

    def close(self):
        pass

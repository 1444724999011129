"""General partitioned (grace) hash join stage: ``outer.Join(inner, ok, ik, result)`` followed by
any program, over inputs of any size, HBM first and pinned host DRAM past the budget.

The fused join (runtime/fused_join.py) covers one idiom only: a Join folded by Sum / Count /
Average into a linear int64 term.  Every other Join (a ToStore of the pairs, a Select of a string
or float result, a GroupBy of the pairs, a float Sum, ...) would otherwise materialise the whole
co-partitioned inputs and every matching pair in HBM at once (gpu/ops.py op_hash_join).  The
reference plans the same operator as HashPartition vertices writing N x M files and a HashJoin
vertex per partition that builds a lookup of its inner partition and streams the outer one
through it (DryadLinqQueryGen.VisitJoin :1419-1609; DryadLinqVertex.HashJoin :852-897,
ParallelHashJoin :6703); partitions are sized so a vertex's inner side fits in memory.  Here the
whole plan idiom

    read(outer) [-> HashPartition -(cross)-> Merge] --.
                                                      +-> Join -> rest of the stage's program
    read(inner) [-> HashPartition -(cross)-> Merge] --'

runs as ONE gang stage:

  * pass A: both inputs are read chunk by chunk (gen://records64, hbm:// column tables, partfile://
    fixed-width record tables decoded on the device) into rows of [key, the fields the result
    selector reads] (column pruning by tracing the selector), hash-routed to their rank over
    xGMI and into hash buckets (ops/grace.GraceHashJoin): buckets that fit ``HbmBudgetBytes``
    stay in HBM, the rest spill to pinned host DRAM;
  * pass B, per bucket (spilled ones streamed back one bucket ahead): a device hash table over
    the smaller side, probed by the other (dr_ht_build / dr_ht_probe_pairs), the pair tables
    gathered, the result selector traced over them, and the rest of the stage's program run on
    that bucket's result table;
  * the bucket results are combined: a decomposable aggregate's partials are folded
    (agg_combine), a partfile:// output is appended bucket by bucket to its part file through
    the native writer (never resident as a whole), anything else is concatenated.

Join keys: one integer field per side (the hash of the grace partition).  Pair order inside a
partition is bucket-major (a partitioned join's order, as in the reference).
"""
from __future__ import annotations

import os
import time

import torch
import torch.distributed as dist

from ..gpu.table import DeviceTable, Shape
from ..io.providers import GenProvider, parse_uri, provider_for
from ..parallel import shuffle
from ..utils.log import get_logger
from . import fused_join as FJ

log = get_logger("grace_stage")

CHUNK_ROWS = 1 << 26
_I64 = torch.int64


class StreamedPart:
    """A partition already written to ``path`` (a tmp part file) by a streaming stage; the output
    commit renames it into place (runtime/gpu_executor._commit_partfile_impl)."""

    def __init__(self, path: str, n: int, nbytes: int, dtype, rows: dict | None = None):
        self.path, self.n, self.nbytes, self.dtype = path, n, nbytes, dtype
        self.rows = rows                  # raw fixed-width rows: {stride, key_off, key_len}


# ------------------------------------------------------------------------------------------------
# input sides: rows of int64 words (floats by bit pattern, narrower ints widened)
class _Side:
    fields: list
    dtypes: list                          # torch dtype per field
    shape: Shape
    n: int

    def chunk(self, a: int, b: int, dev) -> torch.Tensor:          # int64 [b - a, len(fields)]
        raise NotImplementedError

    def table(self, words: torch.Tensor, cols: list) -> DeviceTable:
        """DeviceTable of this side from int64 words [m, 1 + len(cols)] (column 0 = key) holding
        the fields ``cols``; fields the selector never reads are absent."""
        out = {}
        for j, f in enumerate(cols):
            w = words[:, 1 + j]
            dt = self.dtypes[f]
            if dt.itemsize == 8:
                out[self.fields[f]] = w.view(dt)
            elif dt.is_floating_point:              # stored as the float64 bit pattern
                out[self.fields[f]] = w.view(torch.float64).to(dt)
            else:
                out[self.fields[f]] = w.to(dt)
        return DeviceTable(words.shape[0], self.shape, out)


def _as_words(cols: list) -> torch.Tensor:
    ws = []
    for c in cols:
        if c.dtype.itemsize == 8:
            ws.append(c.view(_I64))
        elif c.dtype.is_floating_point:
            ws.append(c.double().view(_I64))
        else:
            ws.append(c.to(_I64))
    return torch.stack(ws, 1)


class _GenSide(_Side):
    def __init__(self, uri, part):
        self.g = FJ._GenRows(uri, part)
        self.fields, self.n = list(self.g.fields), self.g.n
        self.dtypes = [_I64] * len(self.fields)
        self.shape = Shape("tuple", self.fields)

    def chunk(self, a, b, dev):
        return self.g.chunk(a, b, dev)


class _TableSide(_Side):
    def __init__(self, t: DeviceTable):
        self.t, self.n = t, t.n
        self.fields = list(t.shape.fields)
        self.dtypes = [t.cols[f].dtype for f in self.fields]
        self.shape = t.shape

    def chunk(self, a, b, dev):
        return _as_words([self.t.cols[f][a:b] for f in self.fields])


class _PartfileSide(_Side):
    """A partfile:// table of fixed-width records: record ranges read by the native chunked
    reader and decoded on the device (ops/codec.decode)."""

    def __init__(self, path, dtype, lay, width):
        self.path, self.dt, self.width = path, dtype, width
        self.n = os.path.getsize(path) // width
        self.fields = [f[0] for f in lay]
        self.dtypes = [f[1] for f in lay]
        self.shape = None

    def chunk(self, a, b, dev):
        from ..io import reader as RD
        from ..ops import codec as CD
        if b <= a:
            return torch.empty((0, len(self.fields)), dtype=_I64, device=dev)
        buf = RD.read_to_device(self.path, dev, offset=a * self.width, length=(b - a) * self.width)
        t = CD.decode(buf, self.dt)
        if self.shape is None:
            self.shape = t.shape
        return _as_words([t.cols[f] for f in self.fields])

    def table(self, words, cols):
        if self.shape is None:
            self.chunk(0, min(self.n, 1), words.device)
        return _Side.table(self, words, cols)


def _side(read_op, part):
    scheme, path, q = parse_uri(read_op["uri"])
    if scheme == "gen" and path.strip("/") == "records64":
        return _GenSide(read_op["uri"], part)
    if scheme == "hbm":
        ent = provider_for(read_op["uri"]).get(read_op["uri"])
        t = ent["local"].get(part)
        if isinstance(t, DeviceTable) and t.rows is None and not t.strs and t.heap is None and t.cols and \
                all(t.cols[f].dim() == 1 and t.cols[f].dtype in _WORD for f in t.shape.fields):
            return _TableSide(t)
        return None
    if scheme in ("partfile", "file"):
        from ..ops import codec as CD
        prov = provider_for(read_op["uri"])
        if not prov.exists(read_op["uri"]):
            return None
        sch = prov.schema(read_op["uri"]) or {}
        dt = read_op.get("dtype") or sch.get("dtype")
        lay = CD.layout(dt) if dt is not None and sch.get("format", "binary") == "binary" else None
        pf = prov.part_file(read_op["uri"], part) if hasattr(prov, "part_file") else None
        if lay is None or pf is None or any(f[1] not in _WORD for f in lay[0]):
            return None
        return _PartfileSide(pf, dt, lay[0], lay[1])
    return None


_WORD = (torch.int64, torch.int32, torch.int16, torch.int8, torch.uint8, torch.bool, torch.float64, torch.float32)


# ------------------------------------------------------------------------------------------------
# plan idiom
def find(plan, taken=()) -> dict:
    """{join stage id: descriptor} for every Join stage whose inputs are read stages (pointwise, or
    HashPartition -(cross)-> [Merge]) consumed only by it, not already taken by the fused join."""
    st = plan.stages
    out = {}
    for j in st:
        if j.id in taken or not j.ops or j.ops[0]["op"] not in ("hash_join", "merge_join") or len(j.inputs) != 2:
            continue
        if j.ops[0].get("comparer") is not None:
            continue
        sides = []
        for inp in j.inputs:
            m = st[inp.src]
            if inp.kind == "cross":
                if [o["op"] for o in m.ops] != ["read", "hash_partition"] or m.inputs or plan.consumers(m.id) != [j.id]:
                    break
                sides.append((m, None))
                continue
            if inp.kind != "pointwise":
                break
            if [o["op"] for o in m.ops] == ["read"] and not m.inputs and plan.consumers(m.id) == [j.id] \
                    and not m.is_output:
                sides.append((m, None))
                continue
            if [o["op"] for o in m.ops] != ["identity"] or len(m.inputs) != 1 or m.inputs[0].kind != "cross":
                break
            hp = st[m.inputs[0].src]
            if [o["op"] for o in hp.ops] != ["read", "hash_partition"] or hp.inputs:
                break
            if plan.consumers(hp.id) != [m.id] or plan.consumers(m.id) != [j.id]:
                break
            sides.append((hp, m))
        if len(sides) != 2 or sides[0][0].id == sides[1][0].id:
            continue
        if len({j.partitions} | {x.partitions for sd in sides for x in sd if x is not None}) != 1:
            continue
        # the program's leading record-at-a-time operators run per bucket (an aggregate's partial
        # ends that prefix); the rest runs once on the combined buckets
        k = 1
        while k < len(j.ops) and j.ops[k]["op"] in PER_BUCKET:
            k += 1
            if j.ops[k - 1]["op"] == "agg_partial":
                break
        out[j.id] = dict(join=j.id, stages=[x.id for sd in sides for x in sd if x is not None],
                         reads=[sides[0][0].ops[0], sides[1][0].ops[0]], op=j.ops[0],
                         per_bucket=j.ops[1:k], after=j.ops[k:], agg=j.ops[k - 1]["op"] == "agg_partial" if k > 1
                         else False)
    return out


PER_BUCKET = ("select", "where", "long_where", "long_select", "output", "group_partial", "agg_partial")


class _Any:
    """A value that supports every operation: traces which record fields a selector reads."""

    def __getattr__(self, name):
        if name.startswith("__"):
            raise AttributeError(name)
        return self

    def __call__(self, *a, **k):
        return self

    def __getitem__(self, i):
        return self

    def __iter__(self):
        return iter(())

    def __bool__(self):
        return True

    def __index__(self):
        return 0

    def __int__(self):
        return 0

    def __float__(self):
        return 0.0

    def __len__(self):
        return 0

    def __hash__(self):
        return 0


def _binop(name):
    return lambda self, *a: self


for _n in ("add radd sub rsub mul rmul truediv rtruediv floordiv rfloordiv mod rmod pow rpow and rand or ror xor "
           "rxor lshift rlshift rshift rrshift lt le gt ge eq ne neg pos abs invert round").split():
    setattr(_Any, f"__{_n}__", _binop(_n))


class _WholeRecord(Exception):
    pass


class _Rec:
    """A record whose field reads are recorded; any other use of the record itself (returned,
    printed, iterated, passed on) means the selector may read every field."""

    def __init__(self, fields, used):
        self._fields, self._used = list(fields), used

    def _whole(self, *a, **k):
        raise _WholeRecord()

    __repr__ = __str__ = __iter__ = __len__ = __hash__ = __eq__ = __bool__ = _whole

    def __getitem__(self, i):
        if isinstance(i, int) and -len(self._fields) <= i < len(self._fields):
            self._used.add(i % len(self._fields))
            return _Any()
        raise KeyError(i)

    def __getattr__(self, name):
        if name.startswith("_") or name not in self._fields:
            raise AttributeError(name)
        self._used.add(self._fields.index(name))
        return _Any()


def _used_fields(fn, fo, fi):
    """Fields of each side the result selector reads (None: unknown, keep them all)."""
    uo, ui = set(), set()
    try:
        res = fn(_Rec(fo, uo), _Rec(fi, ui))
    except Exception:  # noqa: BLE001
        return None

    def has_rec(x):
        return isinstance(x, _Rec) or isinstance(x, (tuple, list)) and any(has_rec(y) for y in x)
    if has_rec(res):
        return None
    return sorted(uo), sorted(ui)


def plan_local(desc, runner):
    """This rank's half of the vote: the layout, or None when the stage cannot run this way."""
    if not runner.gpu_ok:
        return None
    me, W = runner.world.rank, runner.world.size
    P = runner.plan.stages[desc["join"]].partitions
    parts = [p for p in range(P) if runner.owner(p) == me]
    if not parts:
        return None
    sides = [[_side(r, p) for p in parts] for r in desc["reads"]]
    if any(x is None for sd in sides for x in sd):
        return None
    if any(len({(tuple(x.fields), tuple(map(str, x.dtypes))) for x in sd}) != 1 for sd in sides):
        return None
    fo, fi = sides[0][0].fields, sides[1][0].fields
    op = desc["op"]
    try:
        ko = FJ._key_field(op["outer_key"], 0, fo)
        ki = FJ._key_field(op["inner_key"], 1, fi)
    except FJ.NotLinear as e:
        log.info("join %s: no grace stage (%s)", desc["join"], e)
        return None
    if sides[0][0].dtypes[ko].is_floating_point or sides[1][0].dtypes[ki].is_floating_point:
        return None
    used = _used_fields(op["result"], fo, fi) or (list(range(len(fo))), list(range(len(fi))))
    rows = [sum(x.n for x in sd) for sd in sides]
    return dict(ko=ko, ki=ki, uo=used[0], ui=used[1], rows=rows,
                bytes=rows[0] * 8 * len(fo) + rows[1] * 8 * len(fi))


def vote(desc, runner):
    """Collective: the layout every rank agrees on, when this stage should run as a grace join:
    forced by the ``GraceJoin`` context property (False forbids it), or when the inputs would
    crowd the HBM budget the compiled join materialises them in (inputs x 3: the inputs, their
    shuffled copies and the gathered pairs)."""
    force = runner.ctx._props.get("GraceJoin")
    lay = None if force is False else plan_local(desc, runner)
    W = runner.world.size
    votes = [lay]
    if W > 1:
        votes = [None] * W
        dist.all_gather_object(votes, lay)
    if any(v is None for v in votes) or any((v["ko"], v["ki"], v["uo"], v["ui"]) !=
                                            (votes[0]["ko"], votes[0]["ki"], votes[0]["uo"], votes[0]["ui"])
                                            for v in votes):
        return None
    if force is not True:
        from ..ops.extsort import default_budget
        budget = int(runner.ctx._props.get("HbmBudgetBytes") or default_budget(runner.dev))
        if 3 * max(v["bytes"] for v in votes) <= budget:
            return None
    return votes[0]


# ------------------------------------------------------------------------------------------------
def run(desc, runner, lay) -> dict:
    """Execute the stage on this rank -> {local partition: its output} (see the module doc)."""
    from ..ops import grace as GR
    from ..gpu import ops as G
    from ..gpu import trace as TR
    from . import vertex_ops as V
    w, dev = runner.world, runner.dev
    W, me = w.size, w.rank
    stage = runner.plan.stages[desc["join"]]
    parts = [p for p in range(stage.partitions) if runner.owner(p) == me]
    sides = [[_side(r, p) for p in parts] for r in desc["reads"]]
    keys, used = (lay["ko"], lay["ki"]), (lay["uo"], lay["ui"])
    width = 1 + max(len(used[0]), len(used[1]))              # [key, fields..] padded to one stride
    n_loc = torch.tensor([sum(x.n for x in sd) for sd in sides], dtype=_I64, device=dev)
    n_tot, n_max = n_loc.clone(), n_loc.clone()
    shuffle.all_reduce_(n_tot, "sum", w)
    shuffle.all_reduce_(n_max, "max", w)
    n_tot, n_max = n_tot.tolist(), n_max.tolist()
    build = 0 if n_tot[0] < n_tot[1] else 1
    names = ("O", "I")
    chunk_rows = max(1, min(CHUNK_ROWS, max(n_max)))
    sched = []
    for s_ in (0, 1):                     # the same number of (collective) add_chunk calls everywhere
        lst = [(x, a, min(x.n, a + chunk_rows)) for x in sides[s_] for a in range(0, x.n, chunk_rows)]
        cnt = torch.tensor([len(lst)], dtype=_I64, device=dev)
        shuffle.all_reduce_(cnt, "max", w)
        lst += [(sides[s_][0], 0, 0)] * (int(cnt.item()) - len(lst))
        sched.append(lst)
    grace = GR.GraceHashJoin(w, 8 * width, 0, 8, {"O": -(-n_tot[0] // W), "I": -(-n_tot[1] // W)}, chunk_rows,
                             hbm_budget=runner.ctx._props.get("HbmBudgetBytes"), build=names[build])
    t0 = time.perf_counter()
    sink = _Sink(runner, stage, parts, desc)
    matches = 0
    try:
        for s_ in (0, 1):
            sel = [keys[s_]] + list(used[s_])
            for src, a, b in sched[s_]:
                words = src.chunk(a, b, dev)
                rows = torch.zeros((b - a, width), dtype=_I64, device=dev)
                if b > a:
                    rows[:, : len(sel)] = words[:, sel]
                grace.add_chunk(names[s_], rows.view(torch.uint8).reshape(b - a, 8 * width))
        grace.finish_partitioning()
        t1 = time.perf_counter()
        bname, pname = names[build], names[1 - build]
        proto = [sides[0][0], sides[1][0]]
        vctx = runner._vertex_ctx(stage, parts[0])
        for b, brows, prows in grace.buckets(bname, pname):
            if brows.shape[0] == 0 or prows.shape[0] == 0:
                continue
            po, bo = GR.hash_join_pairs(brows, prows, 0, 8)
            if po.numel() == 0:
                continue
            matches += po.numel()
            oi, ii = (bo, po) if build == 0 else (po, bo)
            orows = (brows if build == 0 else prows).view(_I64).view(-1, width)
            irows = (prows if build == 0 else brows).view(_I64).view(-1, width)
            a_ = proto[0].table(orows.index_select(0, oi), used[0])
            b_ = proto[1].table(irows.index_select(0, ii), used[1])
            data = G._result_table(G._traced(desc["op"]["result"], TR.proxy(a_), TR.proxy(b_)), a_)
            for op in desc["per_bucket"]:
                data = runner._run_op(op, [data], vctx, stage)
            sink.add(data)
        t2 = time.perf_counter()
        stats = grace.stats
    except BaseException:
        # the sink's part writer holds the process-wide writer ring: give it back (and drop the
        # partial part file) before the retry or the fallback stages open a writer of their own
        sink.abort()
        raise
    finally:
        grace.release()
    out = sink.finish(V)
    runner.join_stats = dict(spilled_bytes=stats.spilled_bytes, buckets=stats.buckets, resident=stats.resident,
                             in_hbm=stats.in_hbm, build=names[build], layout=f"{width} x 8-byte words (pruned)",
                             matches=matches, partition_s=round(t1 - t0, 4), join_s=round(t2 - t1, 4),
                             written_bytes=sink.written, kind="grace join stage")
    return out


class _Sink:
    """Where the buckets' results go: folded (decomposable aggregate), appended to the output part
    file (partfile:// output, first local partition), or concatenated."""

    def __init__(self, runner, stage, parts, desc):
        self.runner, self.stage, self.parts, self.desc = runner, stage, parts, desc
        self.agg = desc["agg"]
        self.chunks, self.partials = [], []
        self.writer, self.dtype, self.n, self.written = None, None, 0, 0
        self.stream = False
        if stage.is_output and not self.agg and not desc["after"]:
            scheme, path, _ = parse_uri(stage.output["uri"])
            self.stream = scheme in ("partfile", "file") and runner.ctx.OutputDataCompressionScheme.value == 0
            if self.stream:
                from ..io import partfile as PF
                base = PF.default_base(path)
                os.makedirs(os.path.dirname(base) or ".", exist_ok=True)
                self.tmp = f"{base}.{parts[0]:08X}---{runner.vids[stage.id][parts[0]]}_0_stream.tmp"

    def add(self, data):
        if self.agg:
            self.partials.append(data)
            return
        if self.stream and isinstance(data, DeviceTable):
            from ..ops import codec as CD
            if self.dtype is None:
                self.dtype = _table_dtype(data)
            enc = CD.encode(data, self.dtype) if self.dtype is not None else None
            if enc is not None:
                if self.writer is None:
                    from ..io.writer import PartWriter
                    self.writer = PartWriter(self.tmp, data.device, self.runner.write_stats)
                self.writer.write(enc)
                self.n += data.n
                return
            if self.writer is None:
                self.stream = False
        if self.writer is not None:
            raise RuntimeError("grace join stage: a bucket result could not be encoded like the others")
        self.chunks.append(data)

    def abort(self):
        """An attempt failed mid-stream: stop the writer (its threads, the ring lock) and remove
        the partial part file."""
        w, self.writer = self.writer, None
        if w is not None:
            try:
                w.abort()
            finally:
                try:
                    os.remove(self.tmp)
                except OSError:
                    pass
        self.chunks, self.partials = [], []

    def finish(self, V):
        runner, parts = self.runner, self.parts
        out = {p: None for p in parts}
        if self.agg:
            objs = []
            for x in self.partials:
                objs += x if isinstance(x, list) else x.to_objects()
            spec = next(o for o in self.desc["per_bucket"] if o["op"] == "agg_partial")["spec"]
            vctx = runner._vertex_ctx(self.stage, parts[0])
            folded = V.OPS["agg_combine"](dict(op="agg_combine", spec=spec), [objs], vctx) if objs else \
                runner._run_op(next(o for o in self.desc["per_bucket"] if o["op"] == "agg_partial"),
                               [DeviceTable(0, Shape("scalar", ["v"]), {"v": torch.empty(0, dtype=_I64,
                                                                                   device=runner.dev)})],
                               vctx, self.stage)
            data = folded
            for op in self.desc["after"]:
                data = runner._run_op(op, [data], vctx, self.stage)
            out[parts[0]] = data
            empty = V.OPS["agg_combine"](dict(op="agg_combine", spec=spec), [[]], vctx) if len(parts) > 1 else None
            for p in parts[1:]:
                out[p] = empty
            return out
        if self.writer is not None:
            self.written = self.writer.close()
            out[parts[0]] = StreamedPart(self.tmp, self.n, self.written, self.dtype)
            self.writer = None
        else:
            tabs = [c for c in self.chunks if isinstance(c, DeviceTable)]
            if tabs and len(tabs) == len(self.chunks):
                data = DeviceTable.concat(tabs)
            else:
                from .gpu_executor import _to_objects
                data = [x for c in self.chunks for x in (c if isinstance(c, list) else _to_objects(c))]
            if self.desc["after"]:
                vctx = runner._vertex_ctx(self.stage, parts[0])
                for op in self.desc["after"]:
                    data = runner._run_op(op, [data], vctx, self.stage)
            out[parts[0]] = data
        for p in parts[1:]:                   # the rank's other partitions: empty outputs of the same kind
            x = out[parts[0]]
            if isinstance(x, DeviceTable):
                out[p] = x.slice(0, 0)
            elif self.desc["after"] or not isinstance(x, list):
                vctx = runner._vertex_ctx(self.stage, p)
                data = x.slice(0, 0) if isinstance(x, DeviceTable) else []
                for op in self.desc["after"]:
                    data = runner._run_op(op, [data], vctx, self.stage)
                out[p] = data
            else:
                out[p] = []
        return out


def _table_dtype(t: DeviceTable):
    """Record type of a columnar device table of fixed-width numeric fields (None otherwise)."""
    from .. import types as T
    m = {torch.int64: T.Int64, torch.int32: T.Int32, torch.int16: T.Int16, torch.uint8: T.Byte, torch.int8: T.SByte,
         torch.bool: T.Bool, torch.float64: T.Float64, torch.float32: T.Float32}
    if t.rows is not None or t.heap is not None or t.strs:
        return None
    fields = list(t.shape.fields)
    if any(f not in t.cols or t.cols[f].dim() != 1 or t.cols[f].dtype not in m for f in fields):
        return None
    if t.shape.kind == "scalar" and len(fields) == 1:
        return m[t.cols[fields[0]].dtype]
    if t.shape.kind == "tuple":
        return T.RecordT([(f"Item{i + 1}", m[t.cols[f].dtype]) for i, f in enumerate(fields)], tuple)
    return None

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

from ..gpu.table import DeviceTable, Shape
from ..io.providers import GenProvider, parse_uri, provider_for
from ..parallel import shuffle
from ..utils.log import get_logger
from . import fused_join as FJ

log = get_logger("grace_stage")

CHUNK_ROWS = 1 << 26
_I64 = torch.int64
# widest packed join row the grace partitioner takes (dr_grace_partition: kMaxStride bytes); a
# row of longer strings is not packed: the stage is not chosen (vote) or fails non-retryably
MAX_ROW_BYTES = 512


class StreamedPart:
    """A partition already written to ``path`` (a tmp part file, or a list of them: a partition
    split over several part files) by a streaming stage; the output commit renames it into place
    (runtime/gpu_executor._commit_partfile_impl)."""

    def __init__(self, path: str, n: int, nbytes: int, dtype, rows: dict | None = None, bounds: dict | None = None):
        self.path, self.n, self.nbytes, self.dtype = path, n, nbytes, dtype
        self.rows = rows                  # raw fixed-width rows: {stride, key_off, key_len}
        self.bounds = bounds              # integer columns' {field: [min, max]} when measured


# ------------------------------------------------------------------------------------------------
# input sides: device tables chunk by chunk; packed into rows of int64 words for the grace
# partitioner: word 0 = the join key word, then every field the result selector reads (a fixed-
# width field is one word, floats by bit pattern; a string field is a length word and its bytes
# inline, zero-padded, in S words).  S covers the longest string the ranks voted (a side that
# knows its strings' lengths says so before the stage starts) and at least GraceJoinStringBytes;
# a longer string met while partitioning restarts pass A, on every rank alike, with S widened to
# it (run: no string length aborts the join).
class _Side:
    fields: list
    dtypes: list                          # torch dtype per field, None for a string field
    n: int
    shape: Shape | None = None

    def chunk_table(self, a: int, b: int, dev) -> DeviceTable:
        raise NotImplementedError

    def field_words(self, f: int, S: int) -> int:
        return 1 + S if self.dtypes[f] is None else 1

    def max_string_bytes(self, fields) -> int:
        """Longest string among ``fields`` of this side (0: none of them is a string; -1: not
        known before the data is read)."""
        return 0 if all(self.dtypes[f] is not None for f in fields) else -1

    def table(self, words: torch.Tensor, cols: list, S: int) -> DeviceTable:
        """DeviceTable of this side from packed rows ``words`` [m, width] (word 0 = key word)
        holding the fields ``cols`` in order; fields the selector never reads are absent.  String
        fields point into the rows' own bytes (the gathered pair rows are the string heap)."""
        out, strs = {}, {}
        m, width = words.shape
        pos = 1
        heap = None
        for f in cols:
            name, dt = self.fields[f], self.dtypes[f]
            if dt is None:
                if heap is None:
                    heap = words.contiguous().view(torch.uint8).view(-1)
                base = torch.arange(m, dtype=_I64, device=words.device) * (8 * width)
                out[name] = base + 8 * (pos + 1)
                out[name + "#len"] = words[:, pos].contiguous()
                strs[name] = heap
                pos += 1 + S
                continue
            w = words[:, pos]
            if dt.itemsize == 8:
                out[name] = w.view(dt)
            elif dt.is_floating_point:              # stored as the float64 bit pattern
                out[name] = w.view(torch.float64).to(dt)
            else:
                out[name] = w.to(dt)
            pos += 1
        t = DeviceTable(m, self.shape if self.shape is not None else Shape("tuple", list(self.fields)), out)
        t.strs = strs
        return t


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


def _word(c: torch.Tensor) -> torch.Tensor:
    if c.dtype.itemsize == 8:
        return c.view(_I64)
    if c.dtype.is_floating_point:
        return c.double().view(_I64)
    return c.to(_I64)


class _GenSide(_Side):
    def __init__(self, uri, part):
        self.g = FJ._GenRows(uri, part)
        self.fields, self.n = list(self.g.fields), self.g.n
        self.dtypes = [_I64] * len(self.fields)
        self.shape = Shape("tuple", self.fields)

    def chunk_table(self, a, b, dev):
        w = self.g.chunk(a, b, dev)
        return DeviceTable(b - a, self.shape, {f: w[:, j] for j, f in enumerate(self.fields)})


class _NamesSide(_Side):
    """gen://names: (Name string, V1, V2), generated on the device chunk by chunk."""

    def __init__(self, uri, part):
        from ..models import names as NM
        from ..models.records_cpu import dim_multiplier
        _, _, q = parse_uri(uri)
        self.lo, hi = GenProvider().bounds(uri, part)
        self.n = hi - self.lo
        self.nk, self.seed = int(q.get("keys", 1 << 20)), int(q.get("seed", 0))
        self.dim = dim_multiplier(self.nk) if q.get("mode") == "dim" else 0
        self.name_len = NM.namelen(q)
        self.fields, self.dtypes = list(NM.FIELDS), [None, _I64, _I64]
        self.shape = Shape("tuple", self.fields)

    def max_string_bytes(self, fields) -> int:
        from ..models import names as NM
        return NM.max_name_bytes(self.name_len) if 0 in fields else 0

    def chunk_table(self, a, b, dev):
        from ..models import names as NM
        return NM.device_table(self.lo + a, b - a, self.nk, self.seed, self.dim, dev, self.name_len)


class _TableSide(_Side):
    def __init__(self, t: DeviceTable):
        self.t, self.n = t, t.n
        self.fields = list(t.shape.fields)
        self.dtypes = [None if f in t.strs else t.cols[f].dtype for f in self.fields]
        self.shape = t.shape

    def chunk_table(self, a, b, dev):
        return self.t.slice(a, b)

    def max_string_bytes(self, fields) -> int:
        m = 0
        for f in fields:
            if self.dtypes[f] is None and self.t.n:
                m = max(m, int(self.t.cols[self.fields[f] + "#len"][: self.t.n].max()))
        return m


class _PartfileSide(_Side):
    """A partfile:// table of fixed-width records: record ranges read by the native chunked
    reader and decoded on the device (ops/codec.decode)."""

    def __init__(self, path, dtype, lay, width):
        self.path, self.dt, self.width = path, dtype, width
        self.n = os.path.getsize(path) // width
        self.fields = [f[0] for f in lay]
        self.dtypes = [f[1] for f in lay]
        self.shape = None

    def chunk_table(self, a, b, dev):
        from ..io import reader as RD
        from ..ops import codec as CD
        if b <= a:
            return DeviceTable(0, self.shape or Shape("tuple", self.fields),
                               {f: torch.empty(0, dtype=d, device=dev) for f, d in zip(self.fields, self.dtypes)})
        buf = RD.read_to_device(self.path, dev, offset=a * self.width, length=(b - a) * self.width)
        t = CD.decode(buf, self.dt)
        if self.shape is None:
            self.shape = t.shape
        return t


class _VarPartfileSide(_Side):
    """A partfile:// table of records with string fields: whole index blocks of records read by
    the chunked reader and decoded on the device (ops/codec.decode_var over the part's
    ``.idx`` block index), the part bytes of the chunk being the strings' heap."""

    def __init__(self, path, dtype, vlay, idx):
        self.path, self.dt = path, dtype
        self.n, self.nbytes, self.block, self.offs = idx
        self.fields = [f[0] for f in vlay]
        self.dtypes = [f[1] for f in vlay]
        self.shape = None

    def align(self, rows: int) -> int:
        return max(self.block, rows // self.block * self.block)

    def chunk_table(self, a, b, dev):
        from ..io import reader as RD
        from ..ops import codec as CD
        B = self.block
        if b <= a:
            t = CD.decode_var(torch.empty(0, dtype=torch.uint8, device=dev), self.dt, 0,
                              torch.zeros(0, dtype=_I64, device=dev), B)
            return t
        assert a % B == 0 and (b % B == 0 or b == self.n), (a, b, B)
        lo = int(self.offs[a // B])
        hi = int(self.offs[b // B]) if b < self.n else self.nbytes
        buf = RD.read_to_device(self.path, dev, offset=lo, length=hi - lo)
        bo = torch.from_numpy(self.offs[a // B: -(-b // B)] - lo).to(dev)
        t = CD.decode_var(buf, self.dt, b - a, bo, B)
        if self.shape is None:
            self.shape = t.shape
        return t


def _side(read_op, part):
    scheme, path, q = parse_uri(read_op["uri"])
    if scheme == "gen" and path.strip("/") == "records64":
        return _GenSide(read_op["uri"], part)
    if scheme == "gen" and path.strip("/") == "names":
        return _NamesSide(read_op["uri"], part)
    if scheme == "hbm":
        ent = provider_for(read_op["uri"]).get(read_op["uri"])
        t = ent["local"].get(part)
        if isinstance(t, DeviceTable) and t.rows is None and t.heap is None and t.cols and \
                all(f in t.strs or (t.cols[f].dim() == 1 and t.cols[f].dtype in _WORD) for f in t.shape.fields):
            return _TableSide(t)
        return None
    if scheme in ("partfile", "file"):
        from ..ops import codec as CD
        from ..io import partfile as PF
        prov = provider_for(read_op["uri"])
        if not prov.exists(read_op["uri"]):
            return None
        sch = prov.schema(read_op["uri"]) or {}
        dt = read_op.get("dtype") or sch.get("dtype")
        if dt is None or sch.get("format", "binary") != "binary":
            return None
        pf = prov.part_file(read_op["uri"], part) if hasattr(prov, "part_file") else None
        if pf is None:
            return None
        lay = CD.layout(dt)
        if lay is not None:
            if any(f[1] not in _WORD for f in lay[0]):
                return None
            return _PartfileSide(pf, dt, lay[0], lay[1])
        vlay = CD.var_layout(dt)
        idx = PF.read_index(pf) if vlay is not None and dt not in ("String",) else None
        if vlay is None or idx is None or any(f[1] is not None and f[1] not in _WORD for f in vlay):
            return None
        if len(vlay) == 1:                  # a bare String table (text_table layout): not a record
            return None
        return _VarPartfileSide(pf, dt, [(f[0], f[1]) for f in vlay], idx)
    return None


_WORD = (torch.int64, torch.int32, torch.int16, torch.int8, torch.uint8, torch.bool, torch.float64, torch.float32)


# ------------------------------------------------------------------------------------------------
# join keys: a field or a tuple of fields of each side
class _FieldRef:
    __slots__ = ("i",)

    def __init__(self, i):
        self.i = i


class _KRec:
    def __init__(self, fields):
        self._fields = list(fields)

    def __getitem__(self, i):
        if isinstance(i, int) and -len(self._fields) <= i < len(self._fields):
            return _FieldRef(i % len(self._fields))
        raise KeyError(i)

    def __getattr__(self, name):
        if name.startswith("_") or name not in self._fields:
            raise AttributeError(name)
        return _FieldRef(self._fields.index(name))


def _key_spec(fn, fields):
    """Field indices of a key selector that returns a field or a tuple of fields, else None."""
    try:
        k = fn(_KRec(fields))
    except Exception:  # noqa: BLE001
        return None
    if isinstance(k, _FieldRef):
        return [k.i]
    if isinstance(k, tuple) and k and all(isinstance(x, _FieldRef) for x in k):
        return [x.i for x in k]
    return None


def _key_kinds(side, spec):
    return tuple("str" if side.dtypes[f] is None else "float" if side.dtypes[f].is_floating_point else "int"
                 for f in spec)


def _canon_float(c: torch.Tensor) -> torch.Tensor:
    """float64 with -0.0 -> 0.0 and one NaN (LINQ's Double.Equals: NaN equals NaN, 0.0 == -0.0)."""
    x = c.double() + 0.0
    return torch.where(torch.isnan(x), torch.full_like(x, float("nan")), x)


def _key_word(t: DeviceTable, side, spec, exact: bool) -> torch.Tensor:
    """The join key word of every row of chunk ``t``: the integer key itself or the canonical
    float bits (``exact``), else a 64-bit hash of the key fields (strings by their bytes) whose
    matches are verified field by field after the probe."""
    from ..ops import relational as R
    if exact:
        c = t.cols[side.fields[spec[0]]]
        return _canon_float(c).view(_I64) if c.is_floating_point() else c.to(_I64)
    keys = []
    for f in spec:
        name = side.fields[f]
        if side.dtypes[f] is None:
            keys.append(R.HashKey.string(t.strs[name], t.cols[name], t.cols[name + "#len"]))
        else:
            c = t.cols[name]
            keys.append(R.HashKey.column(_canon_float(c) if c.is_floating_point() else c.to(_I64)))
    _, hs = R.stable_hash_dest(keys, t.n, 0, len(keys) > 1, t.device, want_hash=True)
    return hs


def _pack(t: DeviceTable, side, cols: list, width: int, S: int, kw: torch.Tensor):
    """Rows [m, width] int64: word 0 = kw, then the fields ``cols`` (strings: length + bytes).
    Returns (rows, ok, longest): ok False when a string is longer than S words, and then
    ``longest`` = the chunk's longest string in bytes (0 otherwise)."""
    m = t.n
    rows = torch.zeros((m, width), dtype=_I64, device=kw.device)
    if m == 0:
        return rows, True, 0
    rows[:, 0] = kw
    pos = 1
    ok = True
    lens = []
    for f in cols:
        name = side.fields[f]
        if side.dtypes[f] is None:
            from ..ops import text as TX
            off, ln = t.cols[name].to(_I64), t.cols[name + "#len"].to(_I64)
            rows[:, pos] = ln
            rb = rows.view(torch.uint8).view(m, 8 * width)
            ok = TX.scatter_strings(t.strs[name], off, ln, rb, 8 * (pos + 1), max_len=8 * S) and ok
            lens.append(ln)
            pos += 1 + S
            continue
        rows[:, pos] = _word(t.cols[name])
        pos += 1
    return rows, ok, (0 if ok else max(int(x.max()) for x in lens))


def _verify(orows, irows, oi, ii, lay, S):
    """Pairs whose key fields are equal (hash-keyed joins): each component compared word by word
    (strings: length and inline bytes; floats: as canonical values)."""
    keep = None
    for (of, opos, kind), (inf, ipos, _) in zip(lay["kpos"][0], lay["kpos"][1]):
        if kind == "str":
            a = orows.index_select(0, oi)[:, opos: opos + 1 + S]
            b = irows.index_select(0, ii)[:, ipos: ipos + 1 + S]
            eq = (a == b).all(1)
        elif kind == "float":
            a = orows[:, opos].index_select(0, oi).view(torch.float64)
            b = irows[:, ipos].index_select(0, ii).view(torch.float64)
            eq = (a == b) | (torch.isnan(a) & torch.isnan(b))
        else:
            eq = orows[:, opos].index_select(0, oi) == irows[:, ipos].index_select(0, ii)
        keep = eq if keep is None else keep & eq
    return keep


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
    ko, ki = _key_spec(op["outer_key"], fo), _key_spec(op["inner_key"], fi)
    if ko is None or ki is None or len(ko) != len(ki):
        log.info("join %s: no grace stage (keys are not fields / tuples of fields)", desc["join"])
        return None
    kinds = _key_kinds(sides[0][0], ko)
    if kinds != _key_kinds(sides[1][0], ki):
        return None
    exact = len(ko) == 1 and kinds[0] != "str"
    used = _used_fields(op["result"], fo, fi) or (list(range(len(fo))), list(range(len(fi))))
    uo, ui = list(used[0]), list(used[1])
    if not exact:                         # the key fields travel too: matches are verified
        uo = sorted(set(uo) | set(ko))
        ui = sorted(set(ui) | set(ki))
    rows = [sum(x.n for x in sd) for sd in sides]
    lens = [x.max_string_bytes(u) for sd, u in zip(sides, (uo, ui)) for x in sd]
    return dict(ko=ko, ki=ki, uo=uo, ui=ui, rows=rows, exact=exact, kinds=list(kinds),
                bytes=rows[0] * 8 * len(fo) + rows[1] * 8 * len(fi),
                max_str=-1 if any(x < 0 for x in lens) else max(lens, default=0))


def vote(desc, runner):
    """Collective: the layout every rank agrees on, when this stage should run as a grace join:
    forced by the ``GraceJoin`` context property (False forbids it), or when the inputs would
    crowd the HBM budget the compiled join materialises them in (inputs x 3: the inputs, their
    shuffled copies and the gathered pairs)."""
    force = runner.ctx._props.get("GraceJoin")
    lay = None if force is False else plan_local(desc, runner)
    key = None if lay is None else (lay["ko"], lay["ki"], lay["uo"], lay["ui"], lay["exact"])
    # one tensor all-gather: (ok, digest of the layout, input bytes) of every rank
    agree, vals = shuffle.vote(lay is not None, key, runner.world,
                               values=(0 if lay is None else lay["bytes"], 0 if lay is None else lay["max_str"]))
    if not agree:
        return None
    if force is not True:
        from ..ops.extsort import default_budget
        budget = int(runner.ctx._props.get("HbmBudgetBytes") or default_budget(runner.dev))
        if 3 * max(v[0] for v in vals) <= budget:
            return None
    lens = [v[1] for v in vals]
    out = dict(lay, max_str=-1 if min(lens) < 0 else max(lens))
    if row_bytes(out, runner, desc) > MAX_ROW_BYTES:
        log.info("join %s: no grace stage (strings of %d bytes make rows past %d bytes)", desc["join"],
                 out["max_str"], MAX_ROW_BYTES)
        return None
    return out


def row_bytes(lay, runner, desc) -> int:
    """Bytes of a packed join row for the voted layout (the widest side's: key word, fields,
    strings of ``max(GraceJoinStringBytes, max_str)`` bytes inline)."""
    s_bytes = max(int(runner.ctx._props.get("GraceJoinStringBytes") or 64), int(lay.get("max_str") or 0))
    S = -(-s_bytes // 8)
    me = runner.world.rank
    P = runner.plan.stages[desc["join"]].partitions
    part = next((p for p in range(P) if runner.owner(p) == me), 0)
    words = []
    for r, used in zip(desc["reads"], (lay["uo"], lay["ui"])):
        side = _side(r, part)
        words.append(1 + sum(side.field_words(f, S) for f in used) if side is not None else 1)
    return 8 * max(words)


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
    proto = [sides[0][0], sides[1][0]]
    # inline string bytes: GraceJoinStringBytes, or the longest string the ranks voted
    s_bytes = max(int(runner.ctx._props.get("GraceJoinStringBytes") or 64), int(lay.get("max_str") or 0))

    def layout(S):
        """(row width in words, verification layout) for S inline string words."""
        nwords = [1 + sum(proto[k].field_words(f, S) for f in used[k]) for k in (0, 1)]
        kpos = []        # where each key field sits in the packed rows (verification of hashed matches)
        for k in (0, 1):
            pos, at = 1, {}
            for f in used[k]:
                at[f] = pos
                pos += proto[k].field_words(f, S)
            kpos.append([(f, at.get(f, -1), kind) for f, kind in zip(keys[k], lay["kinds"])])
        return max(nwords), dict(kpos=kpos)            # [key word, fields..] padded to one stride
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
        step = sides[s_][0].align(chunk_rows) if hasattr(sides[s_][0], "align") else chunk_rows
        lst = [(x, a, min(x.n, a + step)) for x in sides[s_] for a in range(0, x.n, step)]
        cnt = torch.tensor([len(lst)], dtype=_I64, device=dev)
        shuffle.all_reduce_(cnt, "max", w)
        lst += [(sides[s_][0], 0, 0)] * (int(cnt.item()) - len(lst))
        sched.append(lst)
    t0 = time.perf_counter()
    sink = _Sink(runner, stage, parts, desc)
    matches = 0
    strings = any(d is None for k in (0, 1) for d in proto[k].dtypes)
    # string lengths unknown before the data is read: every chunk's fit is agreed (a host sync);
    # lengths the ranks voted are covered by S, so no per-chunk agreement is needed
    check = strings and int(lay.get("max_str", -1)) < 0
    widened = 0
    grace = None
    try:
        while True:                       # pass A; again with wider rows if a string did not fit
            S = -(-s_bytes // 8)                                    # inline string words
            width, vlay = layout(S)
            grace = GR.GraceHashJoin(w, 8 * width, 0, 8, {"O": -(-n_tot[0] // W), "I": -(-n_tot[1] // W)},
                                     max(b - a for lst in sched for _, a, b in lst) or 1,
                                     hbm_budget=runner.ctx._props.get("HbmBudgetBytes"), build=names[build])
            need = 0
            for s_ in (0, 1):
                for src, a, b in sched[s_]:
                    t = src.chunk_table(a, b, dev)
                    kw = _key_word(t, src, keys[s_], lay["exact"]) if t.n else torch.empty(0, dtype=_I64, device=dev)
                    rows, ok, longest = _pack(t, src, used[s_], width, S, kw)
                    del t
                    if not ok and not check:
                        raise RuntimeError("grace join: a string longer than the voted maximum (internal)")
                    if check:
                        st = shuffle.gang_status(ok, longest, w)
                        if not all(o for o, _ in st):
                            # a string longer than S words on some rank: every rank widens alike
                            need = max(v for _, v in st)
                            break
                    grace.add_chunk(names[s_], rows.view(torch.uint8).reshape(b - a, 8 * width))
                if need:
                    break
            if not need:
                break
            grace.release()
            grace = None
            s_bytes = -(-need // 64) * 64
            if 8 * layout(-(-s_bytes // 8))[0] > MAX_ROW_BYTES:
                from ..errors import GangAgreementError
                raise GangAgreementError(f"grace join: a {need}-byte string field makes the packed rows wider "
                                         f"than {MAX_ROW_BYTES} bytes", retryable=False)
            widened += 1
            log.info("grace join %s: string of %d bytes, pass A again with %d inline bytes", desc["join"], need, s_bytes)
        grace.finish_partitioning()
        t1 = time.perf_counter()
        bname, pname = names[build], names[1 - build]
        vctx = runner._vertex_ctx(stage, parts[0])
        for b, brows, prows in grace.buckets(bname, pname):
            if brows.shape[0] == 0 or prows.shape[0] == 0:
                continue
            po, bo = GR.hash_join_pairs(brows, prows, 0, 8)
            if po.numel() == 0:
                continue
            oi, ii = (bo, po) if build == 0 else (po, bo)
            orows = (brows if build == 0 else prows).view(_I64).view(-1, width)
            irows = (prows if build == 0 else brows).view(_I64).view(-1, width)
            if not lay["exact"]:           # hash-keyed: keep the pairs whose key fields are equal
                keep = _verify(orows, irows, oi, ii, vlay, S)
                if not bool(keep.all()):
                    oi, ii = oi[keep], ii[keep]
                if oi.numel() == 0:
                    continue
            matches += oi.numel()
            a_ = proto[0].table(orows.index_select(0, oi), used[0], S)
            b_ = proto[1].table(irows.index_select(0, ii), used[1], S)
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
        if grace is not None:
            grace.release()
    out = sink.finish(V)
    runner.join_stats = dict(spilled_bytes=stats.spilled_bytes, buckets=stats.buckets, resident=stats.resident,
                             in_hbm=stats.in_hbm, build=names[build],
                             layout=f"{width} x 8-byte words (pruned{', strings inline' if strings else ''})",
                             string_bytes=8 * S if strings else 0, widened=widened,
                             key="exact" if lay["exact"] else "hashed + verified",
                             matches=matches, partition_s=round(t1 - t0, 4), join_s=round(t2 - t1, 4),
                             written_bytes=sink.written, kind="grace join stage")
    return out


class _Sink:
    """Where the buckets' results go: folded (decomposable aggregate), appended to the output part
    file(s) through runtime/sinks.PartfileSink (partfile:// output, first local partition), or
    concatenated."""

    def __init__(self, runner, stage, parts, desc):
        self.runner, self.stage, self.parts, self.desc = runner, stage, parts, desc
        self.agg = desc["agg"]
        self.chunks, self.partials = [], []
        self.written = 0
        self.pf = None
        if stage.is_output and not self.agg and not desc["after"]:
            from .sinks import PartfileSink
            if PartfileSink.applicable(runner, stage):
                self.pf = PartfileSink(runner, stage, parts[0])

    def add(self, data):
        if self.agg:
            self.partials.append(data)
            return
        if self.pf is not None and isinstance(data, DeviceTable):
            if self.pf.add(data):
                return
            if self.pf.started:
                raise RuntimeError("grace join stage: a bucket result could not be encoded like the others")
            self.pf = None                     # no device encoding: the results are concatenated
        elif self.pf is not None and self.pf.started:
            raise RuntimeError("grace join stage: a bucket result could not be encoded like the others")
        self.chunks.append(data)

    def abort(self):
        """An attempt failed mid-stream: stop the writer (its threads, the ring lock) and remove
        the partial part files."""
        if self.pf is not None:
            self.pf.abort()
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
        if self.pf is not None and self.pf.started:
            out[parts[0]], self.written = self.pf.finish()
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
    """Record type of a columnar device table of fixed-width numeric fields and strings (None
    otherwise)."""
    from .. import types as T
    m = {torch.int64: T.Int64, torch.int32: T.Int32, torch.int16: T.Int16, torch.uint8: T.Byte, torch.int8: T.SByte,
         torch.bool: T.Bool, torch.float64: T.Float64, torch.float32: T.Float32}
    if t.rows is not None or t.heap is not None:
        return None
    fields = list(t.shape.fields)

    def ft(f):
        if f in t.strs:
            return T.String
        return m.get(t.cols[f].dtype) if f in t.cols and t.cols[f].dim() == 1 else None
    types = [ft(f) for f in fields]
    if any(x is None for x in types):
        return None
    if t.shape.kind == "scalar" and len(fields) == 1:
        return types[0]
    if t.shape.kind == "tuple":
        return T.RecordT([(f"Item{i + 1}", x) for i, x in enumerate(types)], tuple)
    return None

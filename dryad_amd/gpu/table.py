"""Device-resident partitions for the GPU executor.

A partition in HBM is a ``DeviceTable``: either

  * ``rows``  — fixed-width row records (``uint8 [n, stride]``), e.g. TeraSort's 100-byte records;
    the key is a byte-string field ``(key_off, key_len)`` compared in memcmp order, or
  * ``cols``  — struct-of-arrays: an ordered dict of equally long 1-D tensors (one per record
    field), with a ``shape`` describing how fields map back to Python records: a scalar, a tuple,
    a dataclass, or a LineRecord-free fixed record, or
  * ``text``  — strings / LineRecords: one UTF-8 byte ``heap`` plus ``off``/``len`` columns (line
    splitting and tokenising happen on the heap in place: ops/text.py).

The DryadLINQ ``channel`` between two vertices on the same GPU is a DeviceTable handed over by
reference (zero copy); across GPUs it is packed into one uint8 row buffer and moved with RCCL.
Output ports of partitioning vertices are *one* permuted table plus port offsets (``Ported``), so
a shuffle never materialises N small tables.
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field

import numpy as np
import torch

from .. import types as T
from . import stats as _stats


@dataclass
class Shape:
    """How columns map to Python records."""
    kind: str                         # "scalar" | "tuple" | "dataclass" | "rows" | "vector" | "text"
    #                                   | "partial" (GroupBy partial aggregates: pytype = PartialMeta)
    fields: list = field(default_factory=list)   # column names in record order
    pytype: object = None
    key_off: int = 0                  # rows: default key field
    key_len: int = 0

    def describe(self):
        if self.kind == "rows":
            return f"rows(key=[{self.key_off},{self.key_off + self.key_len}))"
        return f"{self.kind}({', '.join(self.fields)})"


@dataclass(frozen=True)
class PartialMeta:
    """Layout of a device GroupBy partial-aggregate table: key columns k0..k{nkeys-1} then the
    accumulator columns of each aggregate (a{j}, plus c{j} for averages).  Only plain data, so
    the shape pickles across ranks.  ``key_form`` = "single" | "tuple" (how the host path
    represents the group key).  ``raw``: one row per input record, not aggregated (the partial
    step found almost every key distinct and skipped the fold, gpu/ops.op_group_partial): a count
    without a predicate and an average's count are implicit (1 per row) and have no column."""
    nkeys: int
    kinds: tuple
    key_form: str = "single"
    raw: bool = False


class DeviceTable:
    def __init__(self, n: int, shape: Shape, cols: dict | None = None, rows: torch.Tensor | None = None,
                 heap: torch.Tensor | None = None, strs: dict | None = None):
        self.n = int(n)
        self.shape = shape
        self.cols = cols if cols is not None else {}
        self.rows = rows
        self.heap = heap              # text tables: the byte heap the off/len columns point into
        # string fields of record tables: field -> UTF-8 heap; cols[field] holds the byte offsets
        # and cols[field + "#len"] the byte lengths
        self.strs = strs or {}

    # ------------------------------------------------------------------ construction
    @staticmethod
    def from_rows(rows: torch.Tensor, key_off=0, key_len=None) -> "DeviceTable":
        return DeviceTable(rows.shape[0], Shape("rows", key_off=key_off, key_len=key_len or rows.shape[1]), rows=rows)

    @staticmethod
    def from_columns(cols: dict, shape: Shape) -> "DeviceTable":
        n = next(iter(cols.values())).shape[0] if cols else 0
        return DeviceTable(n, shape, dict(cols))

    @staticmethod
    def empty_like(t: "DeviceTable", n: int = 0) -> "DeviceTable":
        if t.shape.kind == "rows":
            return DeviceTable(n, t.shape, rows=t.rows.new_empty((n, t.rows.shape[1])))
        return DeviceTable(n, t.shape, {k: v.new_empty((n,) + tuple(v.shape[1:])) for k, v in t.cols.items()})

    def col(self, key) -> torch.Tensor:
        """Column by name or by record position (tuple tables built from records name their
        fields Item1..ItemN, device-built ones whatever the producer chose)."""
        if isinstance(key, int):
            return self.cols[self.shape.fields[key]]
        return self.cols[key]

    @property
    def device(self):
        if self.rows is not None:
            return self.rows.device
        for v in self.cols.values():
            return v.device
        return torch.device("cpu")

    @property
    def nbytes(self) -> int:
        if self.rows is not None:
            return self.rows.numel()
        return sum(v.numel() * v.element_size() for v in self.cols.values())

    def row_bytes(self) -> int:
        if self.rows is not None:
            return self.rows.shape[1]
        return sum(_width(v) for v in self.cols.values())

    # ------------------------------------------------------------------ slicing / permutation
    def slice(self, a: int, b: int) -> "DeviceTable":
        if self.rows is not None:
            return DeviceTable(b - a, self.shape, rows=self.rows[a:b])
        cols = {}
        for k, v in self.cols.items():
            cols[k] = v[a:b]
            _stats.inherit(cols[k], v)
        return DeviceTable(b - a, self.shape, cols, heap=self.heap, strs=self.strs)

    def take(self, idx: torch.Tensor) -> "DeviceTable":
        """Gather rows by an int64 index tensor (HIP row gather for row tables)."""
        if self.rows is not None:
            from ..ops import sort as S
            return DeviceTable(idx.shape[0], self.shape, rows=S.gather_rows(self.rows, index=idx.contiguous()))
        return DeviceTable(idx.shape[0], self.shape, {k: v.index_select(0, idx) for k, v in self.cols.items()},
                           heap=self.heap, strs=self.strs)

    def mask(self, m: torch.Tensor) -> "DeviceTable":
        idx = torch.nonzero(m, as_tuple=False).flatten()
        return self.take(idx)

    @staticmethod
    def concat(tables: list) -> "DeviceTable":
        tables = [t for t in tables if t is not None]
        out = DeviceTable._concat(tables)
        if out is not None and out.rows is None and out.heap is None and len(tables) > 1:
            for k, v in out.cols.items():             # column bounds of the pieces (gpu/stats.py);
                if k not in out.strs and all(k in t.cols for t in tables):   # not rebased offsets
                    _stats.union(v, [t.cols[k] for t in tables])
        return out

    @staticmethod
    def _concat(tables: list) -> "DeviceTable":
        if not tables:
            return None
        t0 = tables[0]
        if len(tables) == 1:
            return t0
        adj = DeviceTable._adjacent(tables)
        if adj is not None:
            return adj
        if t0.rows is not None:
            return DeviceTable(sum(t.n for t in tables), t0.shape, rows=torch.cat([t.rows for t in tables]))
        if t0.heap is not None:
            offs, base = [], 0
            for t in tables:
                offs.append(t.cols["off"] + base)
                base += t.heap.shape[0]
            return DeviceTable(sum(t.n for t in tables), t0.shape,
                               {"off": torch.cat(offs), "len": torch.cat([t.cols["len"] for t in tables])},
                               heap=torch.cat([t.heap for t in tables]))
        if t0.strs:
            cols = {k: torch.cat([t.cols[k] for t in tables]) for k in t0.cols}
            strs = {}
            for f in t0.strs:
                offs, base = [], 0
                for t in tables:
                    offs.append(t.cols[f] + base)
                    base += t.strs[f].shape[0]
                cols[f] = torch.cat(offs)
                strs[f] = torch.cat([t.strs[f] for t in tables])
            return DeviceTable(sum(t.n for t in tables), t0.shape, cols, strs=strs)
        return DeviceTable(sum(t.n for t in tables), t0.shape,
                           {k: torch.cat([t.cols[k] for t in tables]) for k in t0.cols})

    @staticmethod
    def _adjacent(tables: list):
        """Tables that are consecutive row slices of one table (e.g. the pieces one exchange
        delivered for a partition): one view instead of a copy."""
        from ..parallel.exchange import _span
        t0 = tables[0]
        if t0.heap is not None and any(t.heap is not t0.heap for t in tables):
            return None
        if any(t.strs.keys() != t0.strs.keys() or any(t.strs[f] is not t0.strs[f] for f in t0.strs) for t in tables):
            return None
        if t0.rows is not None:
            if any(t.rows is None for t in tables):
                return None
            r = _span([t.rows for t in tables])
            return None if r is None else DeviceTable(r.shape[0], t0.shape, rows=r)
        if any(t.rows is not None or t.cols.keys() != t0.cols.keys() for t in tables):
            return None
        cols = {}
        for k in t0.cols:
            v = _span([t.cols[k] for t in tables])
            if v is None:
                return None
            cols[k] = v
        return DeviceTable(sum(t.n for t in tables), t0.shape, cols, heap=t0.heap, strs=t0.strs)

    # ------------------------------------------------------------------ packing for RCCL
    def pack(self) -> torch.Tensor:
        """One uint8 [n, row_bytes] buffer (AoS) so an exchange is a single collective."""
        if self.heap is not None or self.strs:
            raise TypeError("tables with strings are exchanged as records")
        if self.rows is not None:
            return self.rows
        if self.n == 0:                        # (an empty, possibly expanded column has no byte view)
            return torch.empty((0, sum(_width(v) for v in self.cols.values())), dtype=torch.uint8,
                               device=self.device)
        parts = [v.contiguous().view(torch.uint8).reshape(self.n, _width(v)) for v in self.cols.values()]
        if not parts:
            return torch.empty((self.n, 0), dtype=torch.uint8, device=self.device)
        return torch.cat(parts, dim=1) if len(parts) > 1 else parts[0]

    def unpack_like(self, buf: torch.Tensor, n: int) -> "DeviceTable":
        if self.rows is not None:
            return DeviceTable(n, self.shape, rows=buf.reshape(n, self.rows.shape[1]))
        if n == 0:                             # a rank that receives nothing (no byte views of empty slices)
            return DeviceTable(0, self.shape, {k: torch.empty((0,) + tuple(v.shape[1:]), dtype=v.dtype,
                                                              device=buf.device) for k, v in self.cols.items()})
        buf = buf.reshape(n, -1)
        out, off = {}, 0
        for k, v in self.cols.items():
            w = _width(v)
            # a fresh [n, w] buffer: contiguous() / clone() keep a one-row slice's offset and stride,
            # which a byte -> wider dtype view rejects
            piece = torch.empty((n, w), dtype=torch.uint8, device=buf.device)
            piece.copy_(buf[:, off:off + w])
            out[k] = piece.view(v.dtype).reshape((n,) + tuple(v.shape[1:]))
            off += w
        return DeviceTable(n, self.shape, out)

    # ------------------------------------------------------------------ host conversion
    def to_objects(self) -> list:
        if self.n == 0:
            return []
        if self.rows is not None:
            a = self.rows.cpu().numpy()
            return [bytes(r) for r in a]
        if self.heap is not None:
            from ..ops.text import gather_strings
            strs = gather_strings(self.heap, self.cols["off"], self.cols["len"]) if self.heap.is_cuda else \
                _host_strings(self.heap, self.cols["off"], self.cols["len"])
            if self.shape.pytype is not None and self.shape.pytype is not str:
                return [self.shape.pytype(x) for x in strs]
            return strs
        arrs = {k: v.cpu().numpy() for k, v in self.cols.items() if not k.endswith("#len")}
        for f, hp in self.strs.items():
            if hp.is_cuda:
                from ..ops.text import gather_strings
                arrs[f] = _ObjArr(gather_strings(hp, self.cols[f], self.cols[f + "#len"]))
            else:
                arrs[f] = _ObjArr(_host_strings(hp, self.cols[f], self.cols[f + "#len"]))
        sh = self.shape
        if sh.kind == "scalar":
            return arrs[sh.fields[0]].tolist()
        if sh.kind == "vector":
            return [tuple(r) for r in arrs[sh.fields[0]].tolist()]
        lists = [[tuple(r) for r in arrs[f].tolist()] if arrs[f].ndim > 1 else arrs[f].tolist() for f in sh.fields]
        if sh.kind == "tuple":
            return list(zip(*lists))
        if sh.kind == "dataclass":
            return [sh.pytype(*vals) for vals in zip(*lists)]
        if sh.kind == "partial":
            return _partial_objects(sh.pytype, arrs)
        raise ValueError(sh.kind)


def _partial_objects(meta: PartialMeta, arrs: dict) -> list:
    """Partial-aggregate table -> the host path's (key, [acc per aggregate]) pairs
    (runtime/vertex_ops.op_group_partial), so a host group_final can consume device partials."""
    keys = [arrs[f"k{i}"].tolist() for i in range(meta.nkeys)]
    kv = keys[0] if meta.nkeys == 1 and meta.key_form == "single" else list(zip(*keys))
    accs = []
    n = len(keys[0]) if keys else 0
    for j, kind in enumerate(meta.kinds):
        a = arrs[f"a{j}"].tolist() if f"a{j}" in arrs else [1] * n            # raw: implicit count
        if kind == "avg":
            accs.append(list(zip(a, arrs[f"c{j}"].tolist() if f"c{j}" in arrs else [1] * n)))
        elif kind in ("any", "all"):
            accs.append([bool(x) for x in a])
        else:
            accs.append(a)
    return [(k, [acc[i] for acc in accs]) for i, k in enumerate(kv)]


class _ObjArr(list):
    """A list standing in for a numpy column of strings in to_objects."""
    ndim = 1

    def tolist(self):
        return list(self)


def _host_strings(heap, off, ln) -> list:
    b = heap.numpy().tobytes()
    return [b[o:o + n].decode("utf-8", "replace") for o, n in zip(off.tolist(), ln.tolist())]


def text_table(heap: torch.Tensor, off: torch.Tensor, ln: torch.Tensor, pytype=None) -> "DeviceTable":
    """A text (string / LineRecord) table over a byte heap."""
    return DeviceTable(off.shape[0], Shape("text", ["off", "len"], pytype), {"off": off, "len": ln}, heap=heap)


def _width(v: torch.Tensor) -> int:
    """Bytes per record of a column ([n] scalars or [n, d] vectors)."""
    per = 1
    for d in v.shape[1:]:
        per *= d
    return per * v.element_size()


@dataclass
class Ported:
    """A multi-port vertex output: ``table`` grouped by port, bucket i = rows
    [offsets[i], offsets[i+1]) holding port ``order[i]`` (``order`` None: bucket i is port i).
    Partitioning vertices of a multi-rank job number the buckets rank-major (every port of rank 0,
    then rank 1, ...), so each destination rank's rows are one contiguous slice of every column
    and the table itself is the all-to-all send buffer (parallel/exchange.py)."""
    table: DeviceTable
    offsets: list
    order: list | None = None

    def _bucket(self, k: int) -> int:
        if self.order is None:
            return k
        pos = self.__dict__.get("_pos")
        if pos is None:
            pos = {p: i for i, p in enumerate(self.order)}
            self.__dict__["_pos"] = pos
        return pos[k]

    def port(self, k: int) -> DeviceTable:
        i = self._bucket(k)
        return self.table.slice(self.offsets[i], self.offsets[i + 1])

    def port_rows(self, k: int) -> int:
        i = self._bucket(k)
        return self.offsets[i + 1] - self.offsets[i]

    @property
    def nports(self):
        return len(self.offsets) - 1


@dataclass
class PortTables:
    """A multi-port vertex output whose ports are separate tables (ForkTuple ports may hold
    different record types); an empty, untyped port is an empty host list."""
    tables: list

    def port(self, k: int):
        return self.tables[k]

    @property
    def nports(self):
        return len(self.tables)


# ---------------------------------------------------------------------------------------------
_NP_OF = {T.Int32: np.int32, T.Int64: np.int64, T.Float64: np.float64, T.Float32: np.float32, T.Bool: np.bool_,
          T.Int16: np.int16, T.Byte: np.uint8, T.SByte: np.int8, T.UInt16: np.uint16}


def columnar_dtype(dt) -> bool:
    """Can records of this DType live as columns in HBM?"""
    if dt in _NP_OF:
        return True
    if isinstance(dt, T.VectorT):
        return dt.elem in _NP_OF
    if isinstance(dt, T.RecordT):
        return all(t in _NP_OF or t == T.String or (isinstance(t, T.VectorT) and t.elem in _NP_OF)
                   for _, t in dt.fields) and not dt.nullable_fields
    return False


def from_objects(records: list, dt, device) -> DeviceTable | None:
    """Ingress: Python records -> DeviceTable (None if the type is not columnar)."""
    if dt is None:
        dt = T.infer_common_type(records[:1000]) if records else T.Int32
    if dt in (T.LineRecordT, T.String):
        strs = [r.Line if isinstance(r, T.LineRecord) else r for r in records]
        enc = [x.encode("utf-8") for x in strs]
        ln = np.asarray([len(x) for x in enc], dtype=np.int64)
        off = np.concatenate([[0], np.cumsum(ln)[:-1]]).astype(np.int64) if len(enc) else np.zeros(0, np.int64)
        heap = torch.frombuffer(bytearray(b"".join(enc)), dtype=torch.uint8) if enc and ln.sum() else \
            torch.zeros(0, dtype=torch.uint8)
        return text_table(heap.to(device), torch.from_numpy(off).to(device), torch.from_numpy(ln).to(device),
                          T.LineRecord if dt == T.LineRecordT else str)
    if not columnar_dtype(dt):
        return None
    if isinstance(dt, T.VectorT):
        npt = _NP_OF[dt.elem]
        a = np.asarray(records, dtype=npt).reshape(len(records), dt.dim) if records else np.zeros((0, dt.dim), npt)
        return DeviceTable.from_columns({"x": torch.from_numpy(a).to(device)}, Shape("vector", ["x"], dt))
    if dt in _NP_OF:
        a = np.asarray(records, dtype=_NP_OF[dt]) if records else np.zeros(0, _NP_OF[dt])
        return DeviceTable.from_columns({"v": torch.from_numpy(a).to(device)}, Shape("scalar", ["v"]))
    names = [n for n, _ in dt.fields]
    cols, strs = {}, {}
    for i, (n, t) in enumerate(dt.fields):
        if dt.pytype in (None, tuple):
            vals = [r[i] for r in records]
        else:
            vals = [getattr(r, n) for r in records]
        if t == T.String:
            heap, off, ln = _encode_strings(vals)
            strs[n] = heap.to(device)
            cols[n] = off.to(device)
            cols[n + "#len"] = ln.to(device)
            continue
        if isinstance(t, T.VectorT):
            npt = _NP_OF[t.elem]
            a = np.asarray(vals, dtype=npt).reshape(len(vals), t.dim) if vals else np.zeros((0, t.dim), npt)
            cols[n] = torch.from_numpy(a).to(device)
            continue
        cols[n] = torch.from_numpy(np.asarray(vals, dtype=_NP_OF[t]) if vals else np.zeros(0, _NP_OF[t])).to(device)
    kind = "tuple" if dt.pytype in (None, tuple) else "dataclass"
    t = DeviceTable.from_columns(cols, Shape(kind, names, None if kind == "tuple" else dt.pytype))
    t.strs = strs
    return t


def _encode_strings(vals: list):
    enc = [("" if v is None else str(v)).encode("utf-8") for v in vals]
    ln = np.asarray([len(x) for x in enc], dtype=np.int64)
    off = (np.concatenate([[0], np.cumsum(ln)[:-1]]) if len(enc) else np.zeros(0)).astype(np.int64)
    blob = b"".join(enc)
    heap = torch.frombuffer(bytearray(blob), dtype=torch.uint8) if blob else torch.zeros(0, dtype=torch.uint8)
    return heap, torch.from_numpy(off), torch.from_numpy(ln)

"""Record type system: the Python-side equivalent of the .NET types DryadLINQ serializes.

The reference derives a record's wire format from its static .NET type (auto-generated serializers,
LinqToDryad/DryadLinqCodeGen.cs:792-1479; primitive serializers DryadLinqSerialization.cs:41-789).
Python values are dynamically typed, so every dataset carries an explicit ``DType`` (given by the
user on ``FromStore``/``FromEnumerable`` or inferred from values).  Each DType knows:

  * how to encode/decode one value with ``DryadLinqBinaryWriter/Reader`` primitives (byte-compatible)
  * whether it has a fixed width and a columnar (tensor) layout for the GPU executor
  * a total order / hash used by the operators (``key(v)``)

Also defines the public helper types ``LineRecord``, ``Pair``, ``ForkTuple``/``ForkValue``,
``SqlDateTime`` (reference LineRecord.cs, ForkTuple.cs).
"""
from __future__ import annotations

import dataclasses
import datetime as _dt
import decimal as _decimal
import typing
import uuid as _uuid
from dataclasses import dataclass


# ---------------------------------------------------------------------------------------------
# Public record helper types
@dataclass(frozen=True, order=True)
class LineRecord:
    """A line of text (reference LineRecord.cs:34-176): hashes/compares by ``Line``."""
    Line: str = ""

    def __str__(self):
        return self.Line


@dataclass(frozen=True, order=True)
class Pair:
    """Key/value pair (reference ``Pair<K,V>``)."""
    Key: typing.Any = None
    Value: typing.Any = None


@dataclass(frozen=True)
class ForkValue:
    """One-of value produced by a multi-way Fork mapper (reference ForkTuple.cs)."""
    Value: typing.Any = None
    HasValue: bool = False


@dataclass(frozen=True)
class ForkTuple:
    First: ForkValue = ForkValue()
    Second: ForkValue = ForkValue()
    Third: ForkValue = ForkValue()


@dataclass(frozen=True, order=True)
class SqlDateTime:
    DayTicks: int = 0
    TimeTicks: int = 0


# ---------------------------------------------------------------------------------------------
# DTypes
class DType:
    name = "object"
    fixed_width: int | None = None     # bytes, when every value encodes to the same size
    torch_dtype = None                 # columnar element type for the GPU executor
    nullable = False

    def __repr__(self):
        return self.name

    def __eq__(self, other):
        return isinstance(other, DType) and repr(self) == repr(other)

    def __hash__(self):
        return hash(repr(self))

    def encode(self, w, v):  # pragma: no cover - abstract
        raise NotImplementedError

    def decode(self, r):  # pragma: no cover - abstract
        raise NotImplementedError

    def default(self):
        return None


class _Prim(DType):
    def __init__(self, name, width, wfn, rfn, torch_dtype=None, default=0):
        self.name, self.fixed_width, self._w, self._r = name, width, wfn, rfn
        self._torch_name = torch_dtype
        self._default = default

    @property
    def torch_dtype(self):
        if self._torch_name is None:
            return None
        import torch
        return getattr(torch, self._torch_name)

    def encode(self, w, v):
        getattr(w, self._w)(v)

    def decode(self, r):
        return getattr(r, self._r)()

    def default(self):
        return self._default


def _tdt(name):
    return name   # resolved lazily (workers of the CPU executor never import torch)


Byte = _Prim("Byte", 1, "write_byte", "read_byte", _tdt("uint8"))
SByte = _Prim("SByte", 1, "write_sbyte", "read_sbyte", _tdt("int8"))
Bool = _Prim("Bool", 1, "write_bool", "read_bool", _tdt("bool"), False)
Char = _Prim("Char", None, "write_char", "read_char", None, "\0")
Int16 = _Prim("Int16", 2, "write_int16", "read_int16", _tdt("int16"))
UInt16 = _Prim("UInt16", 2, "write_uint16", "read_uint16", _tdt("uint16"))
Int32 = _Prim("Int32", 4, "write_int32", "read_int32", _tdt("int32"))
UInt32 = _Prim("UInt32", 4, "write_uint32", "read_uint32", _tdt("uint32"))
Int64 = _Prim("Int64", 8, "write_int64", "read_int64", _tdt("int64"))
UInt64 = _Prim("UInt64", 8, "write_uint64", "read_uint64", _tdt("uint64"))
Float32 = _Prim("Float32", 4, "write_float", "read_float", _tdt("float32"), 0.0)
Float64 = _Prim("Float64", 8, "write_double", "read_double", _tdt("float64"), 0.0)
Decimal = _Prim("Decimal", 16, "write_decimal", "read_decimal", None, _decimal.Decimal(0))
DateTime = _Prim("DateTime", 8, "write_datetime", "read_datetime", None, _dt.datetime(1, 1, 1))
Guid = _Prim("Guid", 16, "write_guid", "read_guid", None, _uuid.UUID(int=0))
String = _Prim("String", None, "write_string", "read_string", None, "")
SqlDateTimeT = _Prim("SqlDateTime", 8, "write_sqldatetime", "read_sqldatetime", None, SqlDateTime())


class _LineRecordT(DType):
    name = "LineRecord"

    def encode(self, w, v):
        w.write_string(v.Line if isinstance(v, LineRecord) else str(v))

    def decode(self, r):
        return LineRecord(r.read_string())

    def default(self):
        return LineRecord("")


LineRecordT = _LineRecordT()


class Nullable(DType):
    """``Nullable<T>`` of a value type: a bool presence flag then the value when present."""

    def __init__(self, inner: DType):
        self.inner = inner
        self.name = f"Nullable[{inner!r}]"
        self.nullable = True

    def encode(self, w, v):
        w.write_bool(v is not None)
        if v is not None:
            self.inner.encode(w, v)

    def decode(self, r):
        return self.inner.decode(r) if r.read_bool() else None


class ArrayT(DType):
    """1-D array: int32 length then elements (primitive elements as raw little-endian bytes,
    which is what the reference's single WriteRawBytes produces)."""

    def __init__(self, elem: DType):
        self.elem = elem
        self.name = f"Array[{elem!r}]"

    def encode(self, w, v):
        w.write_int32(len(v))
        for x in v:
            self.elem.encode(w, x)

    def decode(self, r):
        n = r.read_int32()
        return [self.elem.decode(r) for _ in range(n)]

    def default(self):
        return []


class VectorT(DType):
    """Fixed-dimension numeric vector (a k-means point, an embedding): the record is a tuple of
    ``dim`` numbers.  Wire format = the reference's serialization of a ``float[]``/``double[]``
    field (int32 length, then raw little-endian elements), so it is byte-compatible with an
    ArrayT of the same element type.  In HBM a vector column is one ``[n, dim]`` tensor."""

    def __init__(self, elem: DType, dim: int):
        self.elem = elem
        self.dim = int(dim)
        self.name = f"Vector[{elem!r},{self.dim}]"
        self.fixed_width = 4 + self.dim * elem.fixed_width if elem.fixed_width else None

    def encode(self, w, v):
        if len(v) != self.dim:
            raise ValueError(f"{self.name}: got {len(v)} elements")
        w.write_int32(self.dim)
        for x in v:
            self.elem.encode(w, x)

    def decode(self, r):
        n = r.read_int32()
        return tuple(self.elem.decode(r) for _ in range(n))

    def default(self):
        return tuple(self.elem.default() for _ in range(self.dim))



def Vector(elem: DType, dim: int) -> VectorT:
    return VectorT(elem, dim)


class RecordT(DType):
    """A user-defined record (dataclass or tuple): fields in declaration order.  If any field is
    a nullable reference type, a BitVector of null flags precedes the fields and null fields are
    skipped (reference DryadLinqCodeGen.cs:1041-1096, BitVector.cs:108-147)."""

    def __init__(self, fields: list[tuple[str, DType]], pytype=None, nullable_fields: set | None = None):
        self.fields = list(fields)
        self.pytype = pytype
        self.nullable_fields = set(nullable_fields or ())
        inner = ", ".join(f"{n}:{t!r}" for n, t in self.fields)
        tn = pytype.__name__ if pytype is not None and pytype is not tuple else "Tuple"
        self.name = f"{tn}({inner})"
        ws = [t.fixed_width for _, t in self.fields]
        self.fixed_width = None if (self.nullable_fields or any(x is None for x in ws)) else sum(ws)

    def _get(self, v, i, n):
        if self.pytype is None or self.pytype is tuple or isinstance(v, tuple):
            return v[i]
        return getattr(v, n)

    def encode(self, w, v):
        if self.nullable_fields:
            bits = bytearray((len(self.fields) + 7) // 8)
            for i, (n, _) in enumerate(self.fields):
                if n in self.nullable_fields and self._get(v, i, n) is None:
                    bits[i // 8] |= 1 << (i % 8)
            ln = len(bits)
            while ln > 0 and bits[ln - 1] == 0:
                ln -= 1
            w.write_compact(ln)
            for b in bits[:ln]:
                w.write_byte(b)
        for i, (n, t) in enumerate(self.fields):
            x = self._get(v, i, n)
            if n in self.nullable_fields and x is None:
                continue
            t.encode(w, x)

    def decode(self, r):
        nulls = set()
        if self.nullable_fields:
            ln = r.read_compact()
            bits = bytes(r.read_byte() for _ in range(ln))
            for i in range(len(self.fields)):
                if i // 8 < ln and bits[i // 8] & (1 << (i % 8)):
                    nulls.add(i)
        vals = []
        for i, (n, t) in enumerate(self.fields):
            vals.append(None if i in nulls else t.decode(r))
        if self.pytype is None or self.pytype is tuple:
            return tuple(vals)
        return self.pytype(*vals)

    def default(self):
        vals = [t.default() for _, t in self.fields]
        return tuple(vals) if self.pytype in (None, tuple) else self.pytype(*vals)


class PickleT(DType):
    """Opaque Python objects (no .NET equivalent): length-prefixed pickle blobs.  Only used on
    intermediate channels of the object executor when a record type cannot be inferred."""
    name = "Pickle"

    def encode(self, w, v):
        import pickle
        b = pickle.dumps(v, protocol=pickle.HIGHEST_PROTOCOL)
        w.write_int32(len(b))
        w.write_raw(b)

    def decode(self, r):
        import pickle
        n = r.read_int32()
        return pickle.loads(r.read_raw(n))


Pickle = PickleT()

PRIMITIVES = {t.name: t for t in [Byte, SByte, Bool, Char, Int16, UInt16, Int32, UInt32, Int64, UInt64, Float32,
                                  Float64, Decimal, DateTime, Guid, String, SqlDateTimeT, LineRecordT]}

_PY_ANNOT = {int: Int64, float: Float64, str: String, bool: Bool, bytes: ArrayT(Byte), LineRecord: LineRecordT,
             _decimal.Decimal: Decimal, _dt.datetime: DateTime, _uuid.UUID: Guid, SqlDateTime: SqlDateTimeT}


def from_annotation(a) -> DType:
    if isinstance(a, DType):
        return a
    if a in _PY_ANNOT:
        return _PY_ANNOT[a]
    origin = typing.get_origin(a)
    if origin is typing.Union:
        args = [x for x in typing.get_args(a) if x is not type(None)]
        if len(args) == 1:
            return Nullable(from_annotation(args[0]))
    if origin in (list, typing.List):
        (e,) = typing.get_args(a) or (object,)
        return ArrayT(from_annotation(e))
    if origin in (tuple, typing.Tuple):
        return RecordT([(f"Item{i + 1}", from_annotation(x)) for i, x in enumerate(typing.get_args(a))], tuple)
    if dataclasses.is_dataclass(a):
        return record_type(a)
    return Pickle


def record_type(cls) -> RecordT:
    hints = typing.get_type_hints(cls)
    fields, nullable = [], set()
    for f in dataclasses.fields(cls):
        t = from_annotation(hints.get(f.name, object))
        if isinstance(t, Nullable) and t.inner in (String, LineRecordT) or isinstance(t, Nullable) and isinstance(
                t.inner, (RecordT, ArrayT)):
            nullable.add(f.name)
            t = t.inner
        fields.append((f.name, t))
    return RecordT(fields, cls, nullable)


VECTOR_MIN_DIM = 16


def infer_type(v) -> DType:
    """Infer the DType of a Python value (ints default to Int32 when they fit, like C# literals)."""
    if isinstance(v, bool):
        return Bool
    if isinstance(v, int):
        return Int32 if -2**31 <= v < 2**31 else Int64
    if isinstance(v, float):
        return Float64
    if isinstance(v, str):
        return String
    if isinstance(v, LineRecord):
        return LineRecordT
    if isinstance(v, _decimal.Decimal):
        return Decimal
    if isinstance(v, _dt.datetime):
        return DateTime
    if isinstance(v, _uuid.UUID):
        return Guid
    if isinstance(v, SqlDateTime):
        return SqlDateTimeT
    if dataclasses.is_dataclass(v) and not isinstance(v, type):
        return record_type(type(v))
    if isinstance(v, tuple) and not hasattr(v, "_fields"):
        # a wide homogeneous float tuple is a vector (k-means points, embeddings), not a record
        if len(v) >= VECTOR_MIN_DIM and all(type(x) is float for x in v):
            return VectorT(Float64, len(v))
        return RecordT([(f"Item{i + 1}", infer_type(x)) for i, x in enumerate(v)], tuple)
    try:
        import numpy as _np
        if isinstance(v, _np.ndarray) and v.ndim == 1:
            et = {_np.dtype("float32"): Float32, _np.dtype("float64"): Float64,
                  _np.dtype("int32"): Int32, _np.dtype("int64"): Int64}.get(v.dtype)
            if et is not None:
                return VectorT(et, v.shape[0])
    except ImportError:  # pragma: no cover
        pass
    return Pickle


_WIDEN = [Int32, Int64, Float64]


def _widen(t: DType, tv: DType) -> DType | None:
    """Common type of two inferred types: numbers widen Int32 -> Int64 -> Float64, tuple records
    widen field by field (a tuple stream whose first key fits 32 bits and later keys do not is
    still an Int64 column); None when they do not combine."""
    if t == tv:
        return t
    if t in _WIDEN and tv in _WIDEN:
        return _WIDEN[max(_WIDEN.index(t), _WIDEN.index(tv))]
    if isinstance(t, RecordT) and isinstance(tv, RecordT) and t.pytype is tv.pytype and \
            len(t.fields) == len(tv.fields) and not t.nullable_fields and not tv.nullable_fields and \
            all(a == b for (a, _), (b, _) in zip(t.fields, tv.fields)):
        fields = []
        for (n, a), (_, b) in zip(t.fields, tv.fields):
            w = _widen(a, b)
            if w is None:
                return None
            fields.append((n, w))
        return RecordT(fields, t.pytype)
    return None


def infer_common_type(values) -> DType:
    """Widen the inferred type over a sample of values (Int32 -> Int64 -> Float64, per field of
    tuple records)."""
    t = None
    for v in values:
        tv = infer_type(v)
        if t is None:
            t = tv
        elif t != tv:
            t = _widen(t, tv)
            if t is None:
                return Pickle
    return t or Int32


# ---------------------------------------------------------------------------------------------
# Declarative type descriptors (the ``.dryadtype`` sidecar of a partfile table).  Plain JSON, like
# the reference's plain-text partfile metadata: reading a table's schema never runs code.  A
# record's Python class is looked up by ``module:qualname`` among modules already imported by the
# reader (never imported on its behalf); an unknown class reads back as tuple records.
def dtype_to_json(dt):
    if dt is None:
        return None
    if isinstance(dt, _Prim) or dt is LineRecordT:
        return {"t": dt.name}
    if isinstance(dt, Nullable):
        return {"t": "Nullable", "inner": dtype_to_json(dt.inner)}
    if isinstance(dt, VectorT):
        return {"t": "Vector", "elem": dtype_to_json(dt.elem), "dim": dt.dim}
    if isinstance(dt, ArrayT):
        return {"t": "Array", "elem": dtype_to_json(dt.elem)}
    if isinstance(dt, RecordT):
        py = None
        if dt.pytype is tuple or dt.pytype is None:
            py = "tuple"
        else:
            py = f"{dt.pytype.__module__}:{dt.pytype.__qualname__}"
        return {"t": "Record", "fields": [[n, dtype_to_json(t)] for n, t in dt.fields],
                "nullable": sorted(dt.nullable_fields), "pytype": py}
    if isinstance(dt, PickleT):
        return {"t": "Pickle"}
    raise TypeError(f"no declarative descriptor for {dt!r}")


def _lookup_class(spec: str):
    import sys
    mod, _, qual = spec.partition(":")
    obj = sys.modules.get(mod)
    for part in qual.split("."):
        if obj is None or part == "<locals>":
            return None
        obj = getattr(obj, part, None)
    return obj if isinstance(obj, type) else None


def dtype_from_json(o):
    if o is None:
        return None
    t = o["t"]
    if t in PRIMITIVES:
        return PRIMITIVES[t]
    if t == "Nullable":
        return Nullable(dtype_from_json(o["inner"]))
    if t == "Vector":
        return VectorT(dtype_from_json(o["elem"]), int(o["dim"]))
    if t == "Array":
        return ArrayT(dtype_from_json(o["elem"]))
    if t == "Record":
        py = o.get("pytype")
        cls = tuple if py in (None, "tuple") else _lookup_class(py)
        fields = [(n, dtype_from_json(x)) for n, x in o["fields"]]
        if cls is None or (cls is not tuple and not dataclasses.is_dataclass(cls)):
            cls = tuple
        return RecordT(fields, cls, set(o.get("nullable") or ()))
    if t == "Pickle":
        return Pickle
    raise ValueError(f"unknown type descriptor {t!r}")

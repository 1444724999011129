"""Vectorised evaluation of user lambdas over HBM columns ("lambdas -> GPU").

The reference compiles C# lambdas into vertex code.  Here a lambda is *called once per partition*
with proxy arguments whose fields are whole device columns (``Col``); Python operators on ``Col``
become tensor operations, so ``lambda r: (r.k % 10, r.v * 2.0)`` evaluates to two new columns with
no per-record Python.  Anything the proxies cannot express (branching on a value, calling
arbitrary Python functions on it, string ops) raises ``NotTraceable`` and the executor runs that
operator on host objects instead (recorded in the job's explain output).
"""
from __future__ import annotations

import dataclasses

import torch

from .table import DeviceTable, Shape


class NotTraceable(Exception):
    pass


def _t(x):
    return x.t if isinstance(x, Col) else x


class Col:
    """A vector value: one tensor element per record."""
    __slots__ = ("t",)

    def __init__(self, t):
        self.t = t

    def __bool__(self):
        raise NotTraceable("data-dependent branch")

    def __iter__(self):
        raise NotTraceable("iteration over a field")

    def __len__(self):
        raise NotTraceable("len() of a field")

    def __index__(self):
        raise NotTraceable("index use of a field")

    def __hash__(self):
        raise NotTraceable("hash of a field")

    def __str__(self):
        raise NotTraceable("str() of a field")

    def __format__(self, spec):
        raise NotTraceable("format() of a field")

    def __getattr__(self, name):
        raise NotTraceable(f"attribute {name} of a scalar field")

    def __getitem__(self, k):
        raise NotTraceable("indexing a scalar field")

    def __neg__(self):
        return Col(-self.t)

    def __pos__(self):
        return self

    def __abs__(self):
        return Col(self.t.abs())

    def __invert__(self):
        return Col(~self.t)

    def __truediv__(self, o):
        return Col(self.t.to(torch.float64) / _t(o))

    def __rtruediv__(self, o):
        return Col(_t(o) / self.t.to(torch.float64))

    def __floordiv__(self, o):
        return Col(torch.div(self.t, _t(o), rounding_mode="floor"))

    def __rfloordiv__(self, o):
        return Col(torch.div(_t(o) if isinstance(o, torch.Tensor) else torch.full_like(self.t, o), self.t,
                             rounding_mode="floor"))

    def __mod__(self, o):
        return Col(torch.remainder(*_promote(self.t, _t(o))))

    def __rmod__(self, o):
        return Col(torch.remainder(torch.full_like(self.t, o), self.t))


def _bin(name, fn, rfn=None, arith=False):
    if arith:
        setattr(Col, f"__{name}__", lambda a, b: Col(fn(*_promote(a.t, _t(b)))))
        if rfn is not None:
            setattr(Col, f"__r{name}__", lambda a, b: Col(rfn(*_promote(a.t, _t(b)))))
        return
    setattr(Col, f"__{name}__", lambda a, b: Col(fn(a.t, _t(b))))
    if rfn is not None:
        setattr(Col, f"__r{name}__", lambda a, b: Col(rfn(a.t, _t(b))))


def _promote(a, b):
    """Arithmetic with a floating operand runs in float64, as the LocalDebug oracle's Python
    floats (and C#'s long * double) do: torch alone would compute int64 column * 1.5 in float32.
    Integer arithmetic runs in int64: narrower columns (an Int32 field of a stored table) would
    wrap where the oracle's Python ints do not."""
    fb = isinstance(b, float) or isinstance(b, torch.Tensor) and b.is_floating_point()
    wide = torch.float64 if a.is_floating_point() or fb else torch.int64
    if a.dtype != wide:
        a = a.to(wide)
    if isinstance(b, torch.Tensor) and b.dtype != wide:
        b = b.to(wide)
    return a, b


_bin("add", lambda a, b: a + b, lambda a, b: b + a, arith=True)
_bin("sub", lambda a, b: a - b, lambda a, b: b - a, arith=True)
_bin("mul", lambda a, b: a * b, lambda a, b: b * a, arith=True)
_bin("pow", lambda a, b: a ** b, lambda a, b: b ** a, arith=True)
_bin("and", lambda a, b: a & b, lambda a, b: b & a)
_bin("or", lambda a, b: a | b, lambda a, b: b | a)
_bin("xor", lambda a, b: a ^ b, lambda a, b: b ^ a)
_bin("lshift", lambda a, b: a << b)
_bin("rshift", lambda a, b: a >> b)
_bin("lt", lambda a, b: a < b)
_bin("le", lambda a, b: a <= b)
_bin("gt", lambda a, b: a > b)
_bin("ge", lambda a, b: a >= b)
_bin("eq", lambda a, b: a == b)
_bin("ne", lambda a, b: a != b)


@dataclasses.dataclass(frozen=True)
class ByteField:
    """A byte-string slice of fixed-width row records (key in memcmp order)."""
    off: int
    length: int


class RowProxy:
    """Proxy for a fixed-width row record: ``r[a:b]`` selects a byte-string field."""

    def __init__(self, table: DeviceTable):
        self._t = table

    def __getitem__(self, k):
        if isinstance(k, slice):
            a, b, st = k.indices(self._t.rows.shape[1])
            if st != 1:
                raise NotTraceable("strided byte slice")
            return ByteField(a, b - a)
        if isinstance(k, int):
            w = self._t.rows.shape[1]
            i = k + w if k < 0 else k
            if not 0 <= i < w:
                raise NotTraceable("row byte index out of range")
            return Col(self._t.rows[:, i].to(torch.int64))     # bytes[i] is an int in 0..255
        raise NotTraceable("row record index")

    def __getattr__(self, name):
        raise NotTraceable(f"attribute {name} of a row record")

    def __bool__(self):
        raise NotTraceable("branch on a record")


class StrCol:
    """A string field of a record table: (heap, offset, length) per record.  Supports ordinal
    comparisons with constants (==, !=, startswith, endswith, `in`) on the device and can be
    projected into a new table; anything else runs on the host."""
    __slots__ = ("heap", "off", "len")

    def __init__(self, heap, off, ln):
        self.heap, self.off, self.len = heap, off, ln

    def _match(self, pat, mode):
        if not isinstance(pat, str):
            raise NotTraceable("string compared with a non-constant")
        from ..ops.text import str_match
        return Col(str_match(self.heap, self.off, self.len, pat, mode))

    def __eq__(self, o):
        return self._match(o, 0)

    def __ne__(self, o):
        return Col(~self._match(o, 0).t)

    def startswith(self, p):
        return self._match(p, 1)

    def endswith(self, p):
        return self._match(p, 2)

    def __contains__(self, p):
        raise NotTraceable("`in` on a string field must produce a column")   # bool() forces a host value

    def __bool__(self):
        raise NotTraceable("branch on a string field")

    def __hash__(self):
        raise NotTraceable("hash of a string field")

    def __len__(self):
        raise NotTraceable("len() of a string field")

    def __getattr__(self, name):
        raise NotTraceable(f"string method {name}")


def _field(t, name):
    if name in t.strs:
        return StrCol(t.strs[name], t.cols[name], t.cols[name + "#len"])
    return Col(t.cols[name])


class RecProxy:
    """Proxy for a columnar tuple / dataclass record."""

    def __init__(self, table: DeviceTable):
        object.__setattr__(self, "_t", table)

    def __getattr__(self, name):
        t = object.__getattribute__(self, "_t")
        if name in t.cols:
            return _field(t, name)
        raise NotTraceable(f"unknown field {name}")

    def __getitem__(self, i):
        t = object.__getattribute__(self, "_t")
        if isinstance(i, int):
            f = t.shape.fields
            if -len(f) <= i < len(f):
                return _field(t, f[i])
        raise NotTraceable("record index")

    def __iter__(self):
        t = object.__getattribute__(self, "_t")
        return iter([_field(t, f) for f in t.shape.fields])

    def __len__(self):
        return len(object.__getattribute__(self, "_t").shape.fields)

    def __bool__(self):
        raise NotTraceable("branch on a record")


def proxy(table: DeviceTable):
    if table.shape.kind in ("text", "vector"):
        raise NotTraceable(f"lambdas over {table.shape.kind} records run on the host")
    if table.shape.kind == "rows":
        return RowProxy(table)
    if table.shape.kind == "scalar":
        return Col(table.cols[table.shape.fields[0]])
    return RecProxy(table)


_IDENTITY_CACHE: dict = {}


def _code_uses_identity(code) -> bool:
    import dis
    import types
    for ins in dis.get_instructions(code):
        if ins.opname == "IS_OP":
            return True
    return any(_code_uses_identity(c) for c in code.co_consts if isinstance(c, types.CodeType))


def uses_identity(fn) -> bool:
    """Does fn (or a function nested in it) compare with ``is`` / ``is not``?  Identity cannot be
    overloaded, so a traced field would compare as one Python object: ``b is True`` would turn
    into a constant instead of a per-record test (reference MiscBugFixTests Bug15159)."""
    code = getattr(fn, "__code__", None)
    if code is None:
        return False
    r = _IDENTITY_CACHE.get(code)
    if r is None:
        r = _IDENTITY_CACHE[code] = _code_uses_identity(code)
    return r


def call(fn, table: DeviceTable, index_base: int | None = None):
    """Evaluate fn over the table's records; returns the raw traced result."""
    if table.n == 0:
        raise NotTraceable("empty partition (evaluated on host)")
    if uses_identity(fn):
        raise NotTraceable("identity comparison (`is`) on a record")
    args = [proxy(table)]
    if index_base is not None:
        args.append(Col(torch.arange(index_base, index_base + table.n, device=table.device, dtype=torch.int64)))
    try:
        return fn(*args)
    except NotTraceable:
        raise
    except (TypeError, AttributeError, RuntimeError) as e:
        raise NotTraceable(f"{type(e).__name__}: {e}")


def _as_col(v, n, device):
    if isinstance(v, Col):
        t = v.t
        if t.dim() == 0:
            t = t.expand(n)
        return t.contiguous()
    if isinstance(v, bool):
        return torch.full((n,), v, dtype=torch.bool, device=device)
    if isinstance(v, int):
        return torch.full((n,), v, dtype=torch.int32 if -2**31 <= v < 2**31 else torch.int64, device=device)
    if isinstance(v, float):
        return torch.full((n,), v, dtype=torch.float64, device=device)
    raise NotTraceable(f"cannot vectorise value of type {type(v).__name__}")


def to_table(res, table: DeviceTable) -> DeviceTable:
    """Turn a traced projection result into a new DeviceTable."""
    n, dev = table.n, table.device
    if isinstance(res, (RecProxy, RowProxy)):
        return table
    if isinstance(res, ByteField):
        if res.off == 0 and res.length == table.rows.shape[1]:
            return table
        return DeviceTable.from_rows(table.rows[:, res.off:res.off + res.length].contiguous())
    if isinstance(res, StrCol):
        from .table import text_table
        return text_table(res.heap, res.off, res.len, str)
    if isinstance(res, (Col, int, float, bool)):
        return DeviceTable.from_columns({"v": _as_col(res, n, dev)}, Shape("scalar", ["v"]))
    if isinstance(res, tuple) and not hasattr(res, "_fields"):
        names = [f"Item{i + 1}" for i in range(len(res))]
        return _record_table(dict(zip(names, res)), Shape("tuple", names), n, dev)
    if dataclasses.is_dataclass(res) and not isinstance(res, type):
        names = [f.name for f in dataclasses.fields(res)]
        return _record_table({k: getattr(res, k) for k in names}, Shape("dataclass", names, type(res)), n, dev)
    raise NotTraceable(f"projection result of type {type(res).__name__}")


def _record_table(vals: dict, shape, n, dev) -> DeviceTable:
    cols, strs = {}, {}
    for k, v in vals.items():
        if isinstance(v, StrCol):
            cols[k], cols[k + "#len"], strs[k] = v.off, v.len, v.heap
        else:
            cols[k] = _as_col(v, n, dev)
    t = DeviceTable.from_columns(cols, shape)
    t.strs = strs
    return t


def eq_key_columns(res, table: DeviceTable):
    """Key columns for equality-only consumers (GroupBy, HashPartition, Join): a string field is
    replaced by its Rabin-64 fingerprint column (ops/fingerprint.py).  Returns (cols, strkeys)
    with strkeys[i] the StrCol behind cols[i] (None for plain columns); callers must verify that
    rows sharing a fingerprint hold equal strings.  Byte-string row keys stay NotTraceable here."""
    if isinstance(res, RecProxy) and table.strs:
        items = [_field(table, f) for f in table.shape.fields]
    elif isinstance(res, StrCol):
        items = [res]
    elif isinstance(res, tuple) and any(isinstance(v, StrCol) for v in res):
        items = list(res)
    else:
        kind, spec = key_columns(res, table)
        if kind != "cols":
            raise NotTraceable("byte-string key")
        return spec, [None] * len(spec)
    from ..ops.fingerprint import rabin_strings
    cols, skeys = [], []
    for v in items:
        if isinstance(v, StrCol):
            cols.append(rabin_strings(v.heap, v.off, v.len))
            skeys.append(v)
        else:
            cols.append(_as_col(v, table.n, table.device))
            skeys.append(None)
    return cols, skeys


def to_mask(res, table: DeviceTable) -> torch.Tensor:
    if isinstance(res, bool):
        return torch.full((table.n,), res, dtype=torch.bool, device=table.device)
    if isinstance(res, Col) and res.t.dtype == torch.bool:
        return res.t
    raise NotTraceable("predicate did not produce a boolean field")


def key_columns(res, table: DeviceTable):
    """Key selector result -> ("bytes", ByteField) | ("cols", [tensors])."""
    if isinstance(res, ByteField):
        return "bytes", res
    if isinstance(res, RowProxy):
        return "bytes", ByteField(table.shape.key_off, table.shape.key_len or table.rows.shape[1])
    if isinstance(res, Col):
        return "cols", [_as_col(res, table.n, table.device)]
    if isinstance(res, RecProxy):
        if table.strs:
            raise NotTraceable("string keys")
        return "cols", [table.cols[f] for f in table.shape.fields]
    if isinstance(res, tuple):
        if any(isinstance(v, StrCol) for v in res):
            raise NotTraceable("string keys")
        return "cols", [_as_col(v, table.n, table.device) for v in res]
    if isinstance(res, StrCol):
        raise NotTraceable("string keys")
    raise NotTraceable(f"key of type {type(res).__name__}")

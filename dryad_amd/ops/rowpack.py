"""Columnar tables as fixed-width sort rows (csrc/kernels/rowpack.hip).

The fine-bucket range-partitioned sort (ops/recordsort.distributed_sort_rows) moves fixed-width
rows keyed by a byte string.  A columnar table sorted by numeric key columns takes the same path:
its rows are packed with the key first in byte-comparable form (big-endian; signed integers with
the sign bit flipped, floats with the sign-magnitude order made unsigned), then the other columns'
raw bytes, the widest first so every field stays aligned; after the exchange the received rows are
unpacked back into columns.  A key that IS an integer column of the table travels only as its key
bytes and is recovered from them (a float key column is also stored raw: -0.0 sorts as +0.0 but
keeps its bits).  Descending order is the sort's own (inverted key windows).

Reference: the reference's ParallelSort / RangePartition order records of any type with a key
selector and comparer (LinqToDryad/DryadLinqVertex.cs:4909-5151, 9330-9335); here a key of at most
10 bytes (one or more numeric columns, e.g. ``OrderBy(r => r.V1)`` or ``(r.A, r.B)``) makes the
record a byte-keyed row.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _lib
from ._lib import c_u32, c_u64, ptr, stream_of

_KIND = {torch.int64: 1, torch.int32: 1, torch.int16: 1, torch.int8: 1, torch.uint8: 3, torch.bool: 3,
         torch.float32: 2, torch.float64: 2}
MAX_KEY_BYTES = 10
MAX_ROW_BYTES = 128
_RP = np.dtype([("ptr", "<u8"), ("base", "<u8"), ("width", "<u4"), ("off", "<u4"), ("kind", "<u4"), ("flags", "<u4"),
                ("shift", "<u4"), ("kbytes", "<u4")])

_lib.register_signatures({
    "dr_rows_pack": (ctypes.c_int, [ctypes.c_void_p, c_u32, c_u64, c_u32, ctypes.c_void_p, ctypes.c_void_p]),
    "dr_rows_unpack": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, c_u32, c_u64, c_u32, ctypes.c_void_p]),
})


@dataclass
class RowLayout:
    rec: int                     # row bytes (a multiple of 4)
    key_len: int                 # key bytes at offset 0
    # (column name or None for a computed key part, dtype, byte offset, kind, pack flag, unpack flag,
    #  base, shift, key bytes)
    fields: list = field(default_factory=list)
    names: list = field(default_factory=list)     # the table's columns, in order


def ordered(x, dtype) -> int:
    """A key value -> its ordered unsigned integer (the kernel's rp_norm)."""
    w = torch.empty(0, dtype=dtype).element_size()
    kind = _KIND[dtype]
    if kind == 2:
        raw = np.array([x], dtype=np.float32 if w == 4 else np.float64).view(np.uint32 if w == 4 else np.uint64)
        v = int(raw[0])
        sign = 1 << (8 * w - 1)
        if v == sign:
            v = 0
        return ((~v) & ((1 << (8 * w)) - 1)) if v & sign else v | sign
    v = int(x)
    if kind == 1:
        return v + (1 << (8 * w - 1))
    return v


def key_bounds(keys: list, n: int) -> list:
    """Per key part (min, max) of its ordered values over the first ``n`` rows as signed int64
    (ordered - 2^63, the form a tensor vote carries), or the neutral (max, min) for no rows."""
    out = []
    for k in keys:
        if n == 0:
            out += [(1 << 63) - 1, -(1 << 63)]
            continue
        v = k[:n].to(torch.uint8) if k.dtype == torch.bool else k[:n]
        mn, mx = torch.aminmax(v)
        out += [ordered(mn.item(), k.dtype) - (1 << 63), ordered(mx.item(), k.dtype) - (1 << 63)]
    return out


def merge_bounds(per_rank: list, parts: int) -> list:
    """Every rank's key_bounds -> the job's [(ordered min, ordered max)] per key part."""
    res = []
    for j in range(parts):
        mn = min(v[2 * j] for v in per_rank)
        mx = max(v[2 * j + 1] for v in per_rank)
        if mn > mx:
            mn = mx = 0
        res.append((mn + (1 << 63), mx + (1 << 63)))
    return res


def plan(table, keys: list, bounds: list | None = None) -> RowLayout | None:
    """The row layout of ``table`` (columnar, fixed-width numeric columns) sorted by the key tensors
    ``keys`` (TR.key_columns "cols") whose job-wide ordered-value bounds are ``bounds`` (merge_bounds;
    None: each part's full width), or None when it does not fit (strings, key parts wider than 10
    bytes together, rows past 128 bytes)."""
    if table.rows is not None or table.heap is not None or table.strs or not table.cols or not keys:
        return None
    n = table.n
    for c in list(table.cols.values()) + list(keys):
        if c.dtype not in _KIND or c.dim() != 1 or c.shape[0] < n or (n > 1 and c.stride(0) != 1):
            return None
    parts = []
    for j, k in enumerate(keys):
        w = k.element_size()
        lo, hi = bounds[j] if bounds is not None else (0, (1 << (8 * w)) - 1)
        bits = max(1, (hi - lo).bit_length())
        parts.append((lo, 64 - bits, -(-bits // 8)))
    kw = sum(p[2] for p in parts)
    if kw > MAX_KEY_BYTES:
        return None
    fields, off = [], 0
    recovered = set()
    for k, (base, shift, kb) in zip(keys, parts):
        name = None
        for cn, cv in table.cols.items():
            if cv.dtype == k.dtype and _KIND[k.dtype] != 2 and cv.data_ptr() == k.data_ptr() and cn not in recovered:
                name = cn
                break
        if name is not None:
            recovered.add(name)
        fields.append((name, k.dtype, off, _KIND[k.dtype], True, name is not None, base, shift, kb))
        off += kb
    raw = [(cn, cv) for cn, cv in table.cols.items() if cn not in recovered]
    widest = max([cv.element_size() for _, cv in raw] + [1])
    off = -(-off // widest) * widest
    for cn, cv in sorted(raw, key=lambda x: -x[1].element_size()):
        w = cv.element_size()
        off = -(-off // w) * w
        fields.append((cn, cv.dtype, off, 0, True, True, 0, 0, 0))
        off += w
    rec = max(12, -(-off // 4) * 4)
    if rec > MAX_ROW_BYTES:
        return None
    return RowLayout(rec=rec, key_len=kw, fields=fields, names=list(table.cols))


def _descs(lay: RowLayout, tensors: list, device) -> torch.Tensor:
    a = np.zeros(len(lay.fields), dtype=_RP)
    for i, ((_, dt, off, kind, pk, up, base, shift, kb), t) in enumerate(zip(lay.fields, tensors)):
        a[i] = (0 if t is None else t.data_ptr(), base, torch.empty(0, dtype=dt).element_size(), off, kind,
                (1 if pk else 0) | (2 if up else 0), shift, kb)
    return torch.from_numpy(a.view(np.uint8).copy()).to(device, non_blocking=False)


def pack(table, keys: list, lay: RowLayout, out: torch.Tensor) -> torch.Tensor:
    """out[:n] := the table's rows in layout ``lay`` (``out``: uint8 [>= n, lay.rec], contiguous)."""
    _lib.require_gpu_tensor(out, "rowpack.pack")
    n = table.n
    assert out.dtype == torch.uint8 and out.shape[0] >= n and out.shape[1] == lay.rec and out.is_contiguous()
    srcs = list(keys) + [table.cols[f[0]] for f in lay.fields[len(keys):]]     # key parts first
    assert len(srcs) == len(lay.fields)
    for t, f in zip(srcs, lay.fields):
        assert t.dtype == f[1] and t.shape[0] >= n
    d = _descs(lay, srcs, out.device)
    _lib.call("dr_rows_pack", ptr(d), c_u32(len(srcs)), c_u64(n), c_u32(lay.rec), ptr(out), stream_of(out))
    _lib.written(out)
    return out[:n]


def unpack(rows: torch.Tensor, lay: RowLayout, mem: torch.Tensor | None = None) -> dict:
    """Columns of the rows ``rows`` (uint8 [m, lay.rec]) -> {name: tensor [m]} in the table's column
    order; placed back to back in ``mem`` (a flat uint8 tensor not overlapping ``rows``) when it is
    large enough, else allocated."""
    _lib.require_gpu_tensor(rows, "rowpack.unpack")
    m = rows.shape[0]
    assert rows.dtype == torch.uint8 and rows.shape[1] == lay.rec and rows.is_contiguous()
    dts = {f[0]: f[1] for f in lay.fields if f[0] is not None and f[5]}
    need = sum(-(-(m * torch.empty(0, dtype=dt).element_size()) // 256) * 256 for dt in dts.values())
    cols, pos = {}, 0
    for name in lay.names:
        dt = dts[name]
        nb = m * torch.empty(0, dtype=dt).element_size()
        if mem is not None and mem.numel() >= need:
            cols[name] = mem[pos: pos + nb].view(dt)
            pos += -(-nb // 256) * 256
        else:
            cols[name] = torch.empty(m, dtype=dt, device=rows.device)
    dst = [cols[f[0]] if f[0] is not None and f[5] else None for f in lay.fields]
    d = _descs(lay, dst, rows.device)
    _lib.call("dr_rows_unpack", ptr(rows), ptr(d), c_u32(len(dst)), c_u64(m), c_u32(lay.rec), stream_of(rows))
    for c in cols.values():
        _lib.written(c)
    return cols

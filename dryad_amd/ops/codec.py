"""Device DryadLinqBinary codec for fixed-width records (csrc/kernels/codec.hip, K14).

``layout(dtype)`` tells whether a record type serialises to a fixed-width byte row (all fields
fixed-width primitives, no null bitmap) and where each field lives; ``decode`` turns the bytes of
a binary part file (already in HBM) into a columnar DeviceTable, ``encode`` turns a columnar
table back into the exact bytes the host encoder (io/binary.py) writes."""
from __future__ import annotations

import ctypes

import torch

from .. import types as T
from . import _lib
from ._lib import c_i32, c_u32, c_u64, ptr, stream_of, vp

_lib.register_signatures({"dr_codec_fixed": (c_i32, [vp, c_u64, c_u32, c_i32, vp, vp, vp, c_i32, vp])})

_TORCH = {T.Byte: torch.uint8, T.SByte: torch.int8, T.Bool: torch.bool, T.Int16: torch.int16,
          T.UInt16: torch.int16, T.Int32: torch.int32, T.UInt32: torch.int32, T.Int64: torch.int64,
          T.UInt64: torch.int64, T.Float32: torch.float32, T.Float64: torch.float64}


def layout(dtype):
    """[(name, torch dtype, offset, size)], width — or None if not fixed-width columnar."""
    if dtype in _TORCH:
        return [("v", _TORCH[dtype], 0, dtype.fixed_width)], dtype.fixed_width
    if isinstance(dtype, T.RecordT) and not dtype.nullable_fields:
        out, off = [], 0
        for name, ft in dtype.fields:
            if ft not in _TORCH:
                return None
            out.append((name, _TORCH[ft], off, ft.fixed_width))
            off += ft.fixed_width
        return out, off
    return None


def _call(rows, n, width, fields, cols, direction):
    nf = len(fields)
    offs = (ctypes.c_uint32 * nf)(*[f[2] for f in fields])
    sizes = (ctypes.c_uint32 * nf)(*[f[3] for f in fields])
    cps = (ctypes.c_void_p * nf)(*[c.data_ptr() for c in cols])
    _lib.call("dr_codec_fixed", ptr(rows), c_u64(n), c_u32(width), nf, offs, sizes, cps, direction, stream_of(rows))


def decode(buf: torch.Tensor, dtype):
    """HBM bytes of a binary part (n * width) -> DeviceTable (None if dtype is not fixed-width)."""
    from ..gpu.table import DeviceTable, Shape
    lay = layout(dtype)
    if lay is None:
        return None
    fields, width = lay
    if buf.numel() % width:
        raise ValueError(f"part size {buf.numel()} is not a multiple of the record width {width}")
    n = buf.numel() // width
    cols = [torch.empty(n, dtype=dt, device=buf.device) for _, dt, _, _ in fields]
    _call(buf, n, width, fields, cols, 0)
    if dtype in _TORCH:
        return DeviceTable.from_columns({"v": cols[0]}, Shape("scalar", ["v"]))
    names = [f[0] for f in fields]
    kind = "tuple" if dtype.pytype in (None, tuple) else "dataclass"
    return DeviceTable.from_columns(dict(zip(names, cols)), Shape(kind, names, None if kind == "tuple" else dtype.pytype))


def encode(table, dtype) -> torch.Tensor | None:
    """Columnar DeviceTable -> HBM bytes in DryadLinqBinary layout (None if not applicable)."""
    lay = layout(dtype)
    if lay is None or table.heap is not None or table.rows is not None:
        return None
    fields, width = lay
    cols = [table.col(i).contiguous() for i in range(len(fields))] if len(table.shape.fields) == len(fields) else None
    if cols is None:
        return None
    cols = [c.to(dt) for c, (_, dt, _, _) in zip(cols, fields)]
    out = torch.empty(table.n * width, dtype=torch.uint8, device=table.device)
    _call(out, table.n, width, fields, cols, 1)
    return out


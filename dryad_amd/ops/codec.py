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
from ..utils.log import get_logger

log = get_logger("codec")

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



# ------------------------------------------------------------------------------------------------
# Variable-length records: strings (+ fixed-width primitives), csrc/kernels/codec.hip.
_lib.register_signatures({
    "dr_varscan_chains": (c_i32, [vp, c_u64, c_u32, c_i32, ctypes.POINTER(c_u32), vp, vp, vp, c_u32, vp]),
    "dr_varscan_fix": (c_i32, [vp, c_u64, c_u32, c_i32, ctypes.POINTER(c_u32), vp, vp, vp, vp, vp, vp, vp]),
    "dr_varscan_select": (c_i32, [c_u64, c_u32, vp, vp, c_u32, vp, vp]),
    "dr_codec_var_decode": (c_i32, [vp, c_u64, vp, c_u64, c_u32, c_u64, c_i32, ctypes.POINTER(c_u32),
                                    ctypes.POINTER(vp), ctypes.POINTER(vp), vp, vp]),
    "dr_codec_var_sizes": (c_i32, [c_u64, c_i32, ctypes.POINTER(c_u32), ctypes.POINTER(vp), ctypes.POINTER(vp),
                                   ctypes.POINTER(vp), vp, vp, vp]),
    "dr_codec_var_encode": (c_i32, [vp, c_u64, c_i32, ctypes.POINTER(c_u32), ctypes.POINTER(vp), ctypes.POINTER(vp),
                                    ctypes.POINTER(vp), vp, vp, vp]),
})

BLOCK = 64        # records per block of a block index (= io/binary.INDEX_BLOCK)

# FieldKind codes of the native codec (csrc/runtime/codec.h)
_KIND = {T.Byte: 0, T.SByte: 1, T.Bool: 2, T.Int16: 3, T.UInt16: 4, T.Int32: 5, T.UInt32: 6, T.Int64: 7,
         T.UInt64: 8, T.Float32: 9, T.Float64: 10, T.String: 14}


def var_layout(dtype):
    """[(name, torch dtype | None for a string, bytes | 0)] of a record type of fixed-width
    primitives and strings (no nullable fields, at least one string), or None."""
    if dtype in (T.String, T.LineRecordT):
        return [("v", None, 0)]
    if isinstance(dtype, T.RecordT) and not dtype.nullable_fields:
        out = []
        for name, ft in dtype.fields:
            if ft == T.String:
                out.append((name, None, 0))
            elif ft in _TORCH:
                out.append((name, _TORCH[ft], ft.fixed_width))
            else:
                return None
        return out if any(f[1] is None for f in out) and len(out) <= 32 else None
    return None


def schema_codes(dtype) -> list | None:
    if dtype in (T.String, T.LineRecordT):
        return [_KIND[T.String]]
    if isinstance(dtype, T.RecordT) and not dtype.nullable_fields and all(ft in _KIND for _, ft in dtype.fields):
        return [_KIND[ft] for _, ft in dtype.fields]
    return None


def block_index_host(data, dtype, block: int = BLOCK):
    """(records, int64 offsets of every ``block``-th record) of a host record stream (native scan)."""
    import numpy as np
    from ..native import runtime
    codes = schema_codes(dtype)
    if codes is None:
        raise ValueError(f"no native schema for {dtype}")
    n, offs = runtime().scan_record_blocks(data, codes, int(block))
    return int(n), np.asarray(offs, dtype=np.int64)


VARSCAN_CHUNK = 4096          # bytes per speculative chain (csrc/kernels/varscan.hip)
LAST_SCAN: dict = {}          # chunks and whether the last device scan stitched on the device alone
VARSCAN_MAX_WALK = 1 << 16    # records a chain's exit walk may take before giving up


def block_index_device(buf: torch.Tensor, dtype, block: int = BLOCK, chunk: int = VARSCAN_CHUNK,
                       debug: dict | None = None):
    """(records, int64 device offsets of every ``block``-th record) of a part in HBM, found on
    the device by speculative per-chunk parses stitched at their sync points
    (csrc/kernels/varscan.hip), or None when the stream is irregular there (a walk that never
    re-synchronises, a record the plausibility checks reject): the caller then scans on the host.
    Two host syncs (the stitch check and the record count); the pointer chase over chunk sync
    points runs on the host only when some walk did not sync in the very next chunk."""
    import numpy as np
    lay = var_layout(dtype)
    if lay is None or not buf.is_cuda or chunk % 32:
        return None
    n = buf.numel()
    dev = buf.device
    if n == 0:
        return 0, torch.empty(0, dtype=torch.int64, device=dev)
    nf = len(lay)
    sizes = (c_u32 * nf)(*[sz for _, _, sz in lay])
    C = int(chunk)
    nch = (n + C - 1) // C
    bits = torch.empty((n + 31) // 32, dtype=torch.int32, device=dev)
    exitp = torch.empty(nch, dtype=torch.int64, device=dev)
    sync = torch.empty(nch, dtype=torch.int64, device=dev)
    st = stream_of(buf)
    _lib.call("dr_varscan_chains", ptr(buf), c_u64(n), c_u32(C), nf, sizes, ptr(bits), ptr(exitp), ptr(sync),
              c_u32(VARSCAN_MAX_WALK), st)
    # a chunk is "regular" when its chain reached its end and its exit walk met the next chunk's
    # chain inside that chunk: then the next chunk's true entry is that sync point.  Only the
    # irregular chunks (normally none) go to the host, which resolves the path around them.
    good = exitp >= 0
    if nch > 1:
        y = sync[:-1]
        good[:-1] &= (y >= 0) & (y < n) & (torch.div(y, C, rounding_mode="floor") ==
                                           torch.arange(1, nch, device=dev))
    good[-1:] &= exitp[-1:] == n
    bad = torch.nonzero(~good).flatten()
    if debug is not None:
        debug.update(exitp=exitp.clone(), sync=sync.clone(), bits=bits.clone(), good=good.clone())
    entry = torch.cat([torch.zeros(1, dtype=torch.int64, device=dev), sync[:-1]])
    on_path = torch.ones(nch, dtype=torch.uint8, device=dev)
    nbad = int(bad.numel())
    LAST_SCAN.update(chunks=nch, irregular=nbad, fast=nbad == 0)
    if nbad:
        bl = bad.cpu().numpy()
        exb, syb = exitp[bad].cpu().numpy(), sync[bad].cpu().numpy()
        covered = 0                                  # chunks below this one are settled
        off, ek, ev = [], [], []                     # off-path chunk ranges, entry overrides
        for c, e, y in zip(bl.tolist(), exb.tolist(), syb.tolist()):
            if c < covered:
                continue                             # off the path: inside an earlier walk
            if e < 0:                                # the stream is irregular on the path
                return None
            if c == nch - 1:
                if e != n:
                    return None
                continue
            if y < 0:
                return None
            k = nch if y == n else y // C            # the walk ran to chunk k (or to the end)
            if k > c + 1:
                off.append(np.arange(c + 1, k, dtype=np.int64))
            if k < nch:
                ek.append(k)
                ev.append(y)
            covered = k
        if off:
            oi = torch.from_numpy(np.concatenate(off)).to(dev)
            entry[oi] = -1
            on_path[oi] = 0
        if ek:
            entry[torch.tensor(ek, device=dev)] = torch.tensor(ev, dtype=torch.int64, device=dev)
    cnt = torch.zeros(nch, dtype=torch.int64, device=dev)
    _lib.call("dr_varscan_fix", ptr(buf), c_u64(n), c_u32(C), nf, sizes, ptr(entry), ptr(on_path), ptr(exitp),
              ptr(sync), ptr(bits), ptr(cnt), st)
    incl = torch.cumsum(cnt, 0)
    total = int(incl[-1].item())
    base = incl - cnt
    offs = torch.empty((total + block - 1) // block, dtype=torch.int64, device=dev)
    if total:
        _lib.call("dr_varscan_select", c_u64(n), c_u32(C), ptr(bits), ptr(base), c_u32(block), ptr(offs), st)
    return total, offs


def block_index(buf: torch.Tensor, dtype, block: int = BLOCK):
    """(records, int64 device offsets of every ``block``-th record, block) of a part of
    variable-length records in HBM, for a part without a (valid) index sidecar: found on the
    device (block_index_device), the host scan (codec.cpp scan_record_blocks) only when the
    device parse reports the stream irregular."""
    import numpy as np
    got = block_index_device(buf, dtype, block) if buf.is_cuda else None
    if got is not None:
        return got[0], got[1], block
    if buf.is_cuda:
        log.info("variable-length part: device boundary scan declined, scanning %d bytes on the host", buf.numel())
    n, offs = block_index_host(buf.cpu().numpy(), dtype, block)
    return n, torch.from_numpy(np.ascontiguousarray(offs)).to(buf.device), block


class DecodeError(RuntimeError):
    pass


def decode_var(buf: torch.Tensor, dtype, n: int, block_off: torch.Tensor, block: int = BLOCK):
    """HBM bytes of a part of variable-length records -> DeviceTable.  ``block_off``: int64
    (device) byte offsets of records 0, block, 2 block, ...  String fields point into ``buf``
    (the part's bytes become the string heap)."""
    from ..gpu.table import DeviceTable, Shape, text_table
    lay = var_layout(dtype)
    if lay is None:
        return None
    dev = buf.device
    cols, lens = [], []
    for _, dt, sz in lay:
        if dt is None:
            cols.append(torch.empty(n, dtype=torch.int64, device=dev))
            lens.append(torch.empty(n, dtype=torch.int64, device=dev))
        else:
            cols.append(torch.empty(n, dtype=dt, device=dev))
            lens.append(None)
    nf = len(lay)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    if n:
        sizes = (c_u32 * nf)(*[sz for _, _, sz in lay])
        cps = (vp * nf)(*[c.data_ptr() for c in cols])
        lps = (vp * nf)(*[(x.data_ptr() if x is not None else 0) for x in lens])
        bo = block_off.to(device=dev, dtype=torch.int64).contiguous()
        _lib.call("dr_codec_var_decode", ptr(buf), c_u64(buf.numel()), ptr(bo), c_u64(bo.numel()), c_u32(block),
                  c_u64(n), nf, sizes, cps, lps, ptr(err), stream_of(buf))
        if int(err.item()):
            raise DecodeError("record stream does not match its block index")
    if dtype in (T.String, T.LineRecordT):
        return text_table(buf, cols[0], lens[0], T.LineRecord if dtype == T.LineRecordT else str)
    names = [f[0] for f in lay]
    out, strs = {}, {}
    for (name, dt, _), c, ln in zip(lay, cols, lens):
        out[name] = c
        if dt is None:
            out[name + "#len"] = ln
            strs[name] = buf
    kind = "tuple" if dtype.pytype in (None, tuple) else "dataclass"
    t = DeviceTable.from_columns(out, Shape(kind, names, None if kind == "tuple" else dtype.pytype))
    t.strs = strs
    return t


def encode_var(table, dtype, block: int = BLOCK, full_offsets: bool = False):
    """Columnar DeviceTable with string fields -> (HBM record-stream bytes, int64 block index on
    the device) in DryadLinqBinary layout, or None if not applicable.  ``full_offsets``: the
    second value is every record's byte offset (a streamed writer builds the block index of the
    concatenated stream from them)."""
    lay = var_layout(dtype)
    if lay is None or table.rows is not None:
        return None
    n = table.n
    dev = table.device
    cols, lens, heaps = [], [], []
    if dtype in (T.String, T.LineRecordT):
        if table.heap is None:
            return None
        cols.append(table.cols["off"].to(torch.int64).contiguous())
        lens.append(table.cols["len"].to(torch.int64).contiguous())
        heaps.append(table.heap)
    else:
        if len(table.shape.fields) != len(lay):
            return None
        for (name, dt, _), fname in zip(lay, table.shape.fields):
            if dt is None:
                if fname not in table.strs:
                    return None
                cols.append(table.cols[fname].to(torch.int64).contiguous())
                lens.append(table.cols[fname + "#len"].to(torch.int64).contiguous())
                heaps.append(table.strs[fname])
            else:
                c = table.cols[fname]
                if c.dtype != dt or c.dim() != 1:
                    c = c.to(dt)
                cols.append(c.contiguous())
                lens.append(None)
                heaps.append(None)
    nf = len(lay)
    nstr = sum(1 for f in lay if f[1] is None)
    sizes = (c_u32 * nf)(*[sz for _, _, sz in lay])
    cps = (vp * nf)(*[c.data_ptr() for c in cols])
    lps = (vp * nf)(*[(x.data_ptr() if x is not None else 0) for x in lens])
    hps = (vp * nf)(*[(h.data_ptr() if h is not None else 0) for h in heaps])
    units = torch.empty(max(nstr * n, 1), dtype=torch.int32, device=dev)
    rsz = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    st = stream_of(rsz)
    if n:
        _lib.call("dr_codec_var_sizes", c_u64(n), nf, sizes, cps, lps, hps, ptr(units), ptr(rsz), st)
    offs = torch.cumsum(rsz[:n], 0)
    total = int(offs[-1].item()) if n else 0
    offs -= rsz[:n]
    out = torch.empty(total, dtype=torch.uint8, device=dev)
    if n:
        _lib.call("dr_codec_var_encode", ptr(out), c_u64(n), nf, sizes, cps, lps, hps, ptr(units), ptr(offs), st)
    return out, (offs if full_offsets else offs[::block].contiguous())

"""Kernels of the shuffle send side (csrc/kernels/channel.hip): stable multi-column bucket scatter
and string-heap compaction.  CPU tensors (gloo tests of the exchange) take the equivalent torch
path; on a GPU the HIP kernels are required (no silent fallback).

Reference: DryadLinqVertex.HashPartition / RangePartition (LinqToDryad/DryadLinqVertex.cs:4788-5151)
write each record to port ``dest``; here one pass moves every column into port-grouped order.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import c_u32, c_u64, vp

_lib.register_signatures({
    "dr_pc_grid": (c_u32, [c_u64, ctypes.POINTER(c_u64)]),
    "dr_pc_count": (ctypes.c_int, [vp, c_u64, vp, vp, c_u32, c_u64, ctypes.c_int, vp]),
    "dr_pc_scatter": (ctypes.c_int, [vp, c_u64, vp, ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(c_u32),
                                     c_u32, vp, c_u32, c_u64, ctypes.c_int, vp]),
    "dr_copy_segments": (ctypes.c_int, [vp, vp, vp, vp, c_u64, vp, vp]),
    "dr_copy_wide": (ctypes.c_int, [vp, vp, c_u64, c_u32, vp]),
})

MAX_COLS = 16


def col_width(t: torch.Tensor) -> int:
    per = t.element_size()
    for d in t.shape[1:]:
        per *= d
    return per


def kernel_ok(cols: list) -> bool:
    """Can dr_pc_scatter move these columns (<= 16, widths 1, 2 or 4k bytes, aligned, contiguous)?"""
    if len(cols) > MAX_COLS:
        return False
    for c in cols:
        w = col_width(c)
        if w == 0 or (w > 2 and w % 4) or not c.is_contiguous() or c.data_ptr() % min(4, max(w, 1)):
            return False
    return True


def _ports(ent: torch.Tensor, n: int) -> torch.Tensor:
    """Bucket of each row: ``ent`` is E128 entries ([n, 2] int64, port in the low byte of [:, 1])
    or one uint8 port per row (the hash partitioner's compact form)."""
    return ent[:n].to(torch.int64) if ent.dtype == torch.uint8 else ent[:n, 1] & 0xFF


def bucket_counts(ent: torch.Tensor, n: int, lut: torch.Tensor | None):
    """Rows per bucket (256 buckets: the row's port mapped through ``lut``) -> int64 [256] on the
    host, plus the device-side workgroup offsets the scatter needs.  ``ent``: E128 entries or
    uint8 ports."""
    if not ent.is_cuda:
        d = _ports(ent, n)
        if lut is not None:
            d = lut.to(torch.int64)[d]
        return torch.bincount(d, minlength=256)[:256], None
    pb = c_u64(0)
    G = int(_lib.lib().dr_pc_grid(c_u64(n), ctypes.byref(pb)))
    counts = torch.zeros(256 * G, dtype=torch.int32, device=ent.device)
    st = _lib.stream_of(ent)
    _lib.call("dr_pc_count", _lib.ptr(ent), c_u64(n), _lib.ptr(lut) if lut is not None else None, _lib.ptr(counts),
              c_u32(G), pb, int(ent.dtype == torch.uint8), st)
    c64 = counts.to(torch.int64)
    del counts
    offs = torch.cumsum(c64, 0)
    offs -= c64
    return c64.view(256, G).sum(1).cpu(), (offs, G, pb.value)


def scatter_columns(ent: torch.Tensor, n: int, cols: list, lut: torch.Tensor | None = None):
    """Stable partition of the first ``n`` rows of ``cols`` by bucket -> (new columns, int64 [256]
    rows per bucket).  Bucket of row i = lut[port of row i] (identity without a LUT); ``ent``:
    E128 entries (port = ent[i, 1] & 0xFF) or uint8 ports."""
    outs = [torch.empty_like(c[:n]) for c in cols]
    if n == 0:
        return outs, torch.zeros(256, dtype=torch.int64)
    if not ent.is_cuda:
        d = _ports(ent, n)
        if lut is not None:
            d = lut.to(torch.int64)[d]
        order = torch.sort(d, stable=True).indices
        for o, c in zip(outs, cols):
            o.copy_(c[:n].index_select(0, order))
        return outs, torch.bincount(d, minlength=256)[:256]
    _lib.require_gpu_tensor(ent, "scatter_columns")
    tot, (offs, G, pb) = bucket_counts(ent, n, lut)
    k = len(cols)
    ins = (vp * k)(*[c.data_ptr() for c in cols])
    ous = (vp * k)(*[o.data_ptr() for o in outs])
    ws = (c_u32 * k)(*[col_width(c) for c in cols])
    _lib.call("dr_pc_scatter", _lib.ptr(ent), c_u64(n), _lib.ptr(lut) if lut is not None else None, ins, ous, ws,
              c_u32(k), _lib.ptr(offs), c_u32(G), c_u64(pb), int(ent.dtype == torch.uint8), _lib.stream_of(ent))
    return outs, tot


def compact_heap(heap: torch.Tensor, off: torch.Tensor, ln: torch.Tensor, sep: int | None = None):
    """Bytes of strings (off[i], ln[i]) of ``heap`` laid out back to back in row order ->
    (new heap, new int64 offsets).  ``sep``: one byte of that value after every string (e.g.
    b'\\n' to turn selected lines into a tokenisable text heap)."""
    ln = ln.to(torch.int64)
    step = ln + 1 if sep is not None else ln
    doff = torch.cumsum(step, 0) - step
    total = int(step.sum()) if ln.numel() else 0
    out = torch.empty(total, dtype=torch.uint8, device=heap.device)
    if total == 0:
        return out, doff
    if not heap.is_cuda:
        sel = torch.repeat_interleave(doff, ln) + torch.arange(int(ln.sum())) - \
            torch.repeat_interleave(torch.cumsum(ln, 0) - ln, ln)
        src = torch.repeat_interleave(off.to(torch.int64), ln) + sel - torch.repeat_interleave(doff, ln)
        out[sel] = heap.index_select(0, src)
    elif int(ln.sum()) > 0:
        off = off.to(torch.int64).contiguous()
        _lib.call("dr_copy_segments", _lib.ptr(heap), _lib.ptr(off), _lib.ptr(ln.contiguous()), _lib.ptr(doff),
                  c_u64(off.shape[0]), _lib.ptr(out), _lib.stream_of(heap))
    if sep is not None:
        out[doff + ln] = sep
    return out, doff


def copy_wide(dst: torch.Tensor, src: torch.Tensor, stream=None, grid: int = 0) -> None:
    """dst <- src by a CU copy kernel on ``stream``.  One side may be page-locked host memory: the
    CUs then read or write it over PCIe through its device mapping, leaving the DMA engines to the
    other direction (dr_copy_wide).  Both tensors contiguous, same byte size, 16-byte aligned."""
    n = src.numel() * src.element_size()
    if dst.numel() * dst.element_size() != n:
        raise ValueError("copy_wide: size mismatch")
    if n == 0:
        return
    if not (dst.is_contiguous() and src.is_contiguous()):
        raise ValueError("copy_wide: contiguous tensors only")
    dev = dst.device if dst.is_cuda else src.device
    if stream is None:
        stream = torch.cuda.current_stream(dev)
    with torch.cuda.device(dev):
        _lib.call("dr_copy_wide", ctypes.c_void_p(_lib.device_address(dst)), ctypes.c_void_p(_lib.device_address(src)),
                  c_u64(n), c_u32(grid), ctypes.c_void_p(stream.cuda_stream))

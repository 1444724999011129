"""Whole-partition aggregates on the device (csrc/kernels/reduce.hip).

The partial stage of Count / LongCount / Sum / Min / Max / Average / Any / All / Contains /
First / Last / Single (reference: the per-partition aggregate operators of DryadLinqVertex.cs:
1673-4697 under the two-stage plan of DryadLinqQueryGen.cs:3384-3395) is one streaming pass over
the partition's HBM columns: up to 8 aggregate slots per pass, each with an optional predicate
mask, folded in registers / LDS and then across workgroups in a fixed order.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import c_i32, c_u64, ptr, stream_of, vp

_lib.register_signatures({
    "dr_reduce_workspace": (c_u64, []),
    "dr_reduce_multi": (c_i32, [c_i32, ctypes.POINTER(c_i32), ctypes.POINTER(c_i32), ctypes.POINTER(vp),
                                ctypes.POINTER(vp), c_u64, vp, vp, vp]),
})

SUM, MIN, MAX, COUNT, FIRST, LAST = range(6)
_VT = {torch.int64: 0, torch.float64: 1, torch.int32: 2, torch.float32: 3, torch.uint8: 4}
_NO_VALUE = 5
_I64_MAX = (1 << 63) - 1
_WS: dict = {}


def _workspace(dev) -> torch.Tensor:
    ws = _WS.get(str(dev))
    if ws is None:
        ws = torch.empty(int(_lib.lib().dr_reduce_workspace()), dtype=torch.uint8, device=dev)
        _WS[str(dev)] = ws
    return ws


def _aligned(t: torch.Tensor) -> torch.Tensor:
    """The kernel reads 8 rows per lane with 16-byte vector loads: columns start 16-byte aligned."""
    t = t.contiguous()
    return t if t.data_ptr() % 16 == 0 else t.clone()


def _value_column(v: torch.Tensor) -> torch.Tensor:
    if v.dtype == torch.bool:
        return _aligned(v).view(torch.uint8)
    if v.dtype not in _VT:
        v = v.to(torch.float64 if v.is_floating_point() else torch.int64)
    return _aligned(v)


def _mask_column(m: torch.Tensor) -> torch.Tensor:
    return _aligned(m if m.dtype == torch.bool else m != 0).view(torch.uint8)


def reduce_multi(n: int, slots: list, device) -> list:
    """``slots``: [(op, values | None, mask | None)] over columns of length ``n`` in HBM.

    Returns one Python value per slot: an int for integer SUM / MIN / MAX and COUNT, a float for
    float SUM / MIN / MAX, the row index for FIRST / LAST (None when no row qualified).  MIN / MAX
    of no rows return the identity (caller checks emptiness)."""
    res = []
    if not slots:
        return res
    ws = _workspace(device)
    for k in range(0, len(slots), 8):
        chunk = slots[k:k + 8]
        m = len(chunk)
        keep, ops, vts, vals, masks, isf = [], [], [], [], [], []
        for op, v, mk in chunk:
            if op in (SUM, MIN, MAX):
                if v is None or v.shape[0] != n:
                    raise ValueError("SUM / MIN / MAX slots need a value column of the partition's length")
                v = _value_column(v)
                keep.append(v)
                vts.append(_VT[v.dtype])
                vals.append(v.data_ptr())
            else:
                vts.append(_NO_VALUE)
                vals.append(0)
            if mk is not None:
                if mk.shape[0] != n:
                    raise ValueError("mask length differs from the partition's length")
                mk = _mask_column(mk)
                keep.append(mk)
                masks.append(mk.data_ptr())
            else:
                masks.append(0)
            ops.append(op)
            isf.append(vts[-1] in (1, 3))
        out = torch.empty(m, dtype=torch.int64, device=device)
        _lib.call("dr_reduce_multi", m, (c_i32 * m)(*ops), (c_i32 * m)(*vts), (vp * m)(*vals), (vp * m)(*masks),
                  c_u64(n), ptr(out), ptr(ws), stream_of(out))
        host = out.cpu()
        ints, floats = host.tolist(), host.view(torch.float64).tolist()
        for j, op in enumerate(ops):
            if op == FIRST:
                res.append(None if ints[j] == _I64_MAX else ints[j])
            elif op == LAST:
                res.append(None if ints[j] < 0 else ints[j])
            else:
                res.append(floats[j] if isf[j] else ints[j])
        del keep
    return res

"""Device Rabin-64 fingerprints (csrc/kernels/fingerprint.hip).

Bit-identical to the host ``Rabin64`` of the native runtime (csrc/runtime/codec.cpp), which
follows the reference's ``Hash64`` (LinqToDryad/Hash64.cs:29-352, classlib DrFPrint.cpp): the
fingerprint of a byte string ``b`` is ``Rabin64().extend(Rabin64().empty(), b)``.

Used as the 64-bit grouping / partitioning key of string fields on the device (GroupBy,
HashPartition and Distinct over strings): equal strings have equal fingerprints, and callers
verify that rows sharing a fingerprint really hold equal bytes, so a collision can never merge
two different keys.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from ._lib import c_i32, c_u32, c_u64, ptr, stream_of, vp

_lib.register_signatures({
    "dr_rabin_strings": (c_i32, [vp, vp, vp, c_u64, vp, c_u64, vp, vp]),
    "dr_rabin_rows": (c_i32, [vp, c_u64, c_u32, c_u32, c_u32, vp, c_u64, vp, vp]),
    "dr_str_pairs_differ": (c_i32, [vp, vp, vp, vp, vp, vp, vp, vp, c_u64, vp, vp]),
})

_TABLES: dict = {}


def _host_rabin():
    from ..native import runtime
    return runtime().Rabin64()


def empty() -> int:
    """Fingerprint of the empty string (the polynomial itself in the reflected representation)."""
    return int(_host_rabin().empty())


def tables(device) -> torch.Tensor:
    """The eight 256-entry slicing tables as one [8*256] int64 device tensor (cached)."""
    key = str(device)
    t = _TABLES.get(key)
    if t is None:
        r = _host_rabin()
        host = np.concatenate([r.table(b) for b in range(8)]).view(np.int64)
        t = torch.from_numpy(host.copy()).to(device)
        _TABLES[key] = t
    return t


def rabin_strings(heap: torch.Tensor, off: torch.Tensor, ln: torch.Tensor) -> torch.Tensor:
    """int64 fingerprint (two's-complement view of the uint64) of each string heap[off:off+len]."""
    n = off.shape[0]
    out = torch.empty(n, dtype=torch.int64, device=off.device)
    if n == 0:
        return out
    _lib.require_gpu_tensor(off, "rabin_strings")
    if heap.numel() == 0:
        heap = torch.zeros(8, dtype=torch.uint8, device=off.device)
    _lib.call("dr_rabin_strings", ptr(heap), ptr(off.contiguous()), ptr(ln.contiguous()), c_u64(n),
              ptr(tables(off.device)), c_u64(empty()), ptr(out), stream_of(off))
    return out


def rabin_rows(rows: torch.Tensor, col: int = 0, width: int | None = None) -> torch.Tensor:
    """int64 fingerprint of each fixed-width slice rows[i, col:col+width]."""
    _lib.require_gpu_tensor(rows, "rabin_rows")
    n, stride = rows.shape
    width = stride - col if width is None else width
    assert 0 <= col and col + width <= stride
    out = torch.empty(n, dtype=torch.int64, device=rows.device)
    if n:
        _lib.call("dr_rabin_rows", ptr(rows), c_u64(n), c_u32(stride), c_u32(col), c_u32(width),
                  ptr(tables(rows.device)), c_u64(empty()), ptr(out), stream_of(rows))
    return out


def strings_differ(a, ia: torch.Tensor | None, b, ib: torch.Tensor) -> bool:
    """True if any string a[ia[i]] differs from b[ib[i]] (ia None = identity).  ``a``/``b`` are
    (heap, off, len) triples; one device round trip."""
    n = ib.shape[0]
    if n == 0:
        return False
    bad = torch.zeros(1, dtype=torch.int32, device=ib.device)
    ha, oa, la = a
    hb, ob, lb = b
    if ha.numel() == 0:
        ha = torch.zeros(8, dtype=torch.uint8, device=ib.device)
    if hb.numel() == 0:
        hb = torch.zeros(8, dtype=torch.uint8, device=ib.device)
    _lib.call("dr_str_pairs_differ", ptr(ha), ptr(oa.contiguous()), ptr(la.contiguous()),
              ptr(None if ia is None else ia.contiguous()), ptr(hb), ptr(ob.contiguous()), ptr(lb.contiguous()),
              ptr(ib.contiguous()), c_u64(n), ptr(bad), stream_of(ib))
    return bool(bad.item())


def rabin_host(data: bytes) -> int:
    """Host twin (native Rabin64) as a signed int64, for tests and the object path."""
    r = _host_rabin()
    v = int(r.extend(r.empty(), data))
    return v - (1 << 64) if v >= (1 << 63) else v


def signed64(v: int) -> int:
    v &= (1 << 64) - 1
    return v - (1 << 64) if v >= (1 << 63) else v


__all__ = ["empty", "tables", "rabin_strings", "rabin_rows", "rabin_host", "signed64", "strings_differ"]

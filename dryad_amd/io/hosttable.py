"""Pinned host tier of the storage hierarchy: fixed-width row tables in page-locked host DRAM.

SURVEY §5.4/§5.7 plan the channel tiers HBM -> pinned host -> disk.  HBM tables
(``hbm://``, gpu/table.DeviceTable) hold what fits on the GPUs; a ``HostRows`` table holds a
partition that does not (the output of an out-of-core sort, a spilled intermediate) in memory the
DMA engines can read and write directly, so PCIe copies run at full rate in both directions
without a bounce buffer.  The reference's equivalent is the spill of sorted runs to temp files in
``ParallelSort`` (LinqToDryad/DryadLinqVertex.cs:9584-9615, FileEnumerable :10733) — here the
"file" is a page-locked host buffer and the runs are range buckets (ops/extsort.py).  Below it,
``HostRows.mapped`` puts a table in a memory-mapped file (the disk tier) for outputs larger than
host memory.
"""
from __future__ import annotations

import torch

_PINNED: dict = {}        # data_ptr -> nbytes of the page-locked tables alive in this process


def is_registered(t: torch.Tensor) -> bool:
    """True if ``t`` lies inside a page-locked HostRows buffer (DMA-able without staging)."""
    p = t.data_ptr()
    return any(a <= p < a + nb for a, nb in _PINNED.items())


class HostRows:
    """``n`` fixed-width rows of ``stride`` bytes in (when a GPU is present) page-locked host memory.

    ``rows`` is a CPU uint8 tensor ``[n, stride]``; records read back as ``bytes`` objects like the
    rows of a device row table (gpu/table.DeviceTable.to_objects)."""

    def __init__(self, n: int, stride: int, key_off: int = 0, key_len: int | None = None, pinned: bool | None = None):
        self.n, self.stride = int(n), int(stride)
        self.key_off, self.key_len = key_off, key_len or stride
        if pinned is None:
            pinned = torch.cuda.is_available()
        self._buf = None
        if pinned and self.n * self.stride > 0:
            from ..ops._lib import PinnedHostBuffer
            self._buf = PinnedHostBuffer((self.n, self.stride))
            self.rows = self._buf.tensor
            _PINNED[self.rows.data_ptr()] = self.n * self.stride
        else:
            self.rows = torch.empty((self.n, self.stride), dtype=torch.uint8)
        self.pinned = self._buf is not None

    @staticmethod
    def mapped(path: str, n: int, stride: int, key_off: int = 0, key_len: int | None = None) -> "HostRows":
        """A table backed by a memory-mapped file (the disk tier below pinned DRAM): the page cache
        holds what is in use and writes the rest back, so the table may exceed host memory.  The
        file (``path``) stays when the table is released; PCIe copies to and from it are staged
        by the driver (pageable memory)."""
        import numpy as np
        h = HostRows.__new__(HostRows)
        h.n, h.stride = int(n), int(stride)
        h.key_off, h.key_len = key_off, key_len or stride
        h._buf, h.pinned, h.path = None, False, path
        if h.n * h.stride == 0:
            open(path, "wb").close()
            h._mm, h.rows = None, torch.empty((h.n, h.stride), dtype=torch.uint8)
        else:
            h._mm = np.memmap(path, dtype=np.uint8, mode="w+", shape=(h.n, h.stride))
            h.rows = torch.from_numpy(h._mm)
        return h

    def flush(self):
        """Write a mapped table's dirty pages back to its file (no-op for DRAM tables)."""
        mm = getattr(self, "_mm", None)
        if mm is not None:
            mm.flush()

    @staticmethod
    def from_tensor(rows: torch.Tensor, key_off: int = 0, key_len: int | None = None, pinned: bool | None = None):
        """Copy a [n, stride] uint8 tensor (host or device) into a new host table."""
        h = HostRows(rows.shape[0], rows.shape[1], key_off, key_len, pinned)
        if h.n:
            h.rows.copy_(rows)
        return h

    def view(self, n: int) -> "HostRows":
        """A non-owning table over the first ``n`` rows (reusing a preallocated output)."""
        v = HostRows.__new__(HostRows)
        v.n, v.stride, v.key_off, v.key_len = int(n), self.stride, self.key_off, self.key_len
        v._buf, v.rows, v.pinned = None, self.rows[:n], self.pinned
        v._mm, v.path = getattr(self, "_mm", None), getattr(self, "path", None)
        return v

    @property
    def nbytes(self) -> int:
        return self.n * self.stride

    def slice(self, a: int, b: int) -> torch.Tensor:
        return self.rows[a:b]

    def to_objects(self) -> list:
        if self.n == 0:
            return []
        a = self.rows.numpy()
        return [bytes(r) for r in a]

    def release(self):
        if getattr(self, "_mm", None) is not None:
            self._mm.flush()
            self._mm = None
        if self._buf is not None:
            _PINNED.pop(self.rows.data_ptr(), None)
            self._buf.release()
            self._buf = None
        self.rows = None
        self.n = 0

    def __len__(self):
        return self.n


class TieredRows:
    """A row table split across tiers in row order: ``segments`` = [rows tensor [k, stride]], each
    a host tensor (pinned / mapped HostRows storage) or a device (HBM) tensor.  The hybrid
    out-of-core sort (ops/extsort.py, ``resident=True``) returns one: the range buckets that fit the
    HBM budget stay sorted in HBM, the rest sit in host DRAM, so only the overflow crosses PCIe."""

    def __init__(self, segments: list, stride: int, key_off: int = 0, key_len: int | None = None, owners=()):
        self.segments = [s for s in segments if s is not None and s.shape[0] > 0]
        self.stride = int(stride)
        self.key_off, self.key_len = key_off, key_len or stride
        self.n = sum(int(s.shape[0]) for s in self.segments)
        self._owners = list(owners)           # HostRows / device tensors keeping the storage alive

    @property
    def nbytes(self) -> int:
        return self.n * self.stride

    @property
    def device_rows(self) -> int:
        return sum(int(s.shape[0]) for s in self.segments if s.is_cuda)

    @property
    def host_rows(self) -> int:
        return self.n - self.device_rows

    def to_objects(self) -> list:
        out = []
        for s in self.segments:
            a = s.cpu().numpy() if s.is_cuda else s.numpy()
            out += [bytes(r) for r in a]
        return out

    def release(self):
        for o in self._owners:
            if hasattr(o, "release"):
                o.release()
        self._owners, self.segments, self.n = [], [], 0

    def __len__(self):
        return self.n


class HostColumns:
    """A columnar table (fixed-width columns, no string heaps) in page-locked host DRAM, built piece
    by piece: the ``host://`` result of a streamed stage whose output outgrows HBM
    (runtime/sinks.HostSink; a streamed Distinct / GroupBy result, runtime/stream_agg.py).  Each
    piece is one device table's columns copied out by DMA into leased pinned buffers
    (ops/_lib.pinned_lease: exact-size, reused across jobs).  Read back whole (``to_device``),
    piece by piece (``device_pieces``, the chunk source of a later streamed stage) or as records."""

    def __init__(self, shape):
        self.shape = shape
        self.pieces = []               # [(n, {column: pinned tensor [n, ...]}, [leases])]
        self.bounds = []               # per piece: {column: (lo, hi)} of the columns that had them
        self.n = 0

    def append(self, t) -> None:
        from ..ops._lib import pinned_lease
        if t.rows is not None or t.heap is not None or t.strs:
            raise ValueError("HostColumns holds fixed-width columnar tables")
        if t.n == 0:
            return
        from ..gpu import stats as GST
        cols, leases = {}, []
        self.bounds.append({k: b for k, b in ((k, GST.known(v)) for k, v in t.cols.items()) if b is not None})
        for k, v in t.cols.items():
            src = v[: t.n]
            if not src.is_cuda:                 # a CPU run: plain host memory
                cols[k] = src.clone()
                continue
            ls = pinned_lease(tuple(src.shape), src.dtype)
            ls.tensor.copy_(src, non_blocking=True)
            cols[k] = ls.tensor
            leases.append(ls)
        self.pieces.append((t.n, cols, leases))
        self.n += t.n

    @property
    def nbytes(self) -> int:
        return sum(v.numel() * v.element_size() for _, cols, _ in self.pieces for v in cols.values())

    def columns(self) -> list:
        return list(self.pieces[0][1]) if self.pieces else list(self.shape.fields)

    def device_pieces(self, device, max_rows: int | None = None):
        """Yield the table as device tables of at most ``max_rows`` rows, in row order."""
        from ..gpu import stats as GST
        from ..gpu.table import DeviceTable
        for i, (n, cols, _) in enumerate(self.pieces):
            step = n if not max_rows else max(1, int(max_rows))
            bnd = self.bounds[i] if i < len(self.bounds) else {}
            for a in range(0, n, step):
                b = min(n, a + step)
                t = DeviceTable(b - a, self.shape, {k: v[a:b].to(device, non_blocking=True) for k, v in cols.items()})
                for k, (lo, hi) in bnd.items():       # the bounds the piece's columns had on the device
                    GST.set_bounds(t.cols[k], lo, hi)
                yield t

    def to_device(self, device):
        from ..gpu.table import DeviceTable
        if not self.pieces:
            return DeviceTable(0, self.shape, {})
        from ..gpu import stats as GST
        names = self.columns()
        cols = {}
        for k in names:                           # piece by piece into one device column (no host copy)
            first = self.pieces[0][1][k]
            dst = torch.empty((self.n,) + tuple(first.shape[1:]), dtype=first.dtype, device=device)
            a = 0
            for n, c, _ in self.pieces:
                dst[a: a + n].copy_(c[k], non_blocking=True)
                a += n
            cols[k] = dst
        t = DeviceTable(self.n, self.shape, cols)
        for k in names:                           # bounds every piece knew: their union
            bs = [b.get(k) for b in self.bounds]
            if bs and len(bs) == len(self.pieces) and all(x is not None for x in bs):
                GST.set_bounds(t.cols[k], min(x[0] for x in bs), max(x[1] for x in bs))
        return t

    def to_objects(self) -> list:
        from ..gpu.table import DeviceTable
        if torch.cuda.is_available():
            torch.cuda.synchronize()            # the pieces' DMAs are complete
        out = []
        for n, cols, _ in self.pieces:
            out += DeviceTable(n, self.shape, dict(cols)).to_objects()
        return out

    def release(self):
        for _, _, leases in self.pieces:
            for ls in leases:
                ls.release()
        self.pieces, self.bounds, self.n = [], [], 0

    def __len__(self):
        return self.n

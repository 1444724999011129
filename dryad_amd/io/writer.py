"""HBM -> file: a part file written by the native ChunkWriter (csrc/runtime/partwriter.cpp:
writer threads pwrite() 64 MB chunks out of a ring of page-locked host buffers, pre-extending the
file in 256 MB steps) while the next chunks are DMA'd out of HBM on a copy stream, so PCIe
transfers and the page-cache / disk writes overlap.  Replaces device -> pageable ``cpu()`` ->
``tobytes()`` -> Python ``write`` (a full host copy of the partition and a serial write).
Reference: the overlapped native channel writer,
DryadVertex/VertexHost/system/channel/src/channelbuffernativewriter.cpp (256 MB extends at :35).
"""
from __future__ import annotations

import ctypes
import threading
import time
from collections import deque

import torch

CHUNK = 64 << 20
SLOTS = 16         # 1 GB of pinned ring: enough chunks in flight for every writer thread
THREADS = 12       # page-cache copies run at ~3-4 GB/s per pwrite thread (4 threads: 12.3 GB/s,
#                    profiles/r4/stored.log)
MAPPED = False     # True: threads copy into shared mappings of the file instead of pwrite().  On
#                    the MI355X box that fills the page cache at 3.5-6.3 GB/s against pwrite's
#                    11.5-12.6 GB/s (profiles/r4/filewrite_ab.log), so pwrite stays the default

_RING = None
_RING_LOCK = threading.Lock()


def _ring():
    """The process's pinned staging ring for writes (registered once; reused by every writer)."""
    global _RING
    with _RING_LOCK:
        if _RING is None:
            if torch.cuda.is_available():
                from ..ops._lib import PinnedHostBuffer
                _RING = [PinnedHostBuffer((CHUNK,)) for _ in range(SLOTS)]
            else:                    # no GPU: plain host buffers (host sources only)
                _RING = [_HostBuffer(CHUNK) for _ in range(SLOTS)]
        return _RING


class _HostBuffer:
    def __init__(self, n):
        self.tensor = torch.empty(n, dtype=torch.uint8)


class WriteStats:
    def __init__(self):
        self.bytes = 0
        self.seconds = 0.0

    @property
    def gbps(self) -> float:
        return self.bytes / 1e9 / self.seconds if self.seconds else 0.0


class PartWriter:
    """Append device (or host) byte tensors to a new file; ``close()`` returns the byte count.
    One writer per process at a time owns the ring (``with PartWriter(...) as w``).  ``path`` may
    be a list of paths: ``write(data, file=i)`` then appends to file i (a streamed partitioning
    stage writes every output partition at once; ``close()`` returns the byte counts)."""

    def __init__(self, path, device=None, stats: WriteStats | None = None):
        from ..native import runtime
        self.multi = isinstance(path, (list, tuple))
        self.path = path
        self.stats = stats
        self.t0 = time.perf_counter()
        self.ring = _ring()
        _RING_LOCK.acquire()
        try:
            ptrs = [b.tensor.data_ptr() for b in self.ring]
            self.w = runtime().ChunkWriter(list(path), ptrs, THREADS) if self.multi else \
                runtime().ChunkWriter(path, ptrs, THREADS, mapped=MAPPED)
        except Exception:
            _RING_LOCK.release()
            raise
        self.dev = torch.device(device) if device is not None else None
        self.cs = torch.cuda.Stream(self.dev) if self.dev is not None and self.dev.type == "cuda" else None
        self.off = 0
        self.offs = [0] * (len(path) if self.multi else 1)
        self.pending = deque()           # (slot, event, file offset, bytes, file): D2H copies in flight
        self.closed = False

    def __enter__(self):
        return self

    def __exit__(self, et, e, tb):
        if et is None:
            self.close()
        else:
            self.abort()

    def _submit_done(self, block: bool):
        while self.pending and (block or self.pending[0][1] is None or self.pending[0][1].query()):
            slot, ev, off, n, f = self.pending.popleft()
            if ev is not None:
                ev.synchronize()
            self.w.submit(slot, off, n, f)

    def write(self, data, file: int = 0) -> None:
        """Append ``data`` (to file ``file`` of a multi-file writer): a contiguous device or host
        tensor (its bytes), or a bytes-like object."""
        from ..ops import _lib
        if not isinstance(data, torch.Tensor):
            data = torch.frombuffer(bytearray(data), dtype=torch.uint8) if len(data) else torch.empty(0, dtype=torch.uint8)
        flat = data.reshape(-1).view(torch.uint8)
        n = flat.numel()
        if n == 0:
            return
        dev_src = flat.is_cuda
        if dev_src:
            if self.cs is None:
                self.dev = flat.device
                self.cs = torch.cuda.Stream(self.dev)
            self.cs.wait_stream(torch.cuda.current_stream(flat.device))
            flat.record_stream(self.cs)          # the caller may drop it while its DMAs are in flight
        piece = min(CHUNK, self.ring[0].tensor.numel())        # the ring may predate a CHUNK change
        for a in range(0, n, piece):
            m = min(piece, n - a)
            self._submit_done(block=False)
            while len(self.pending) > SLOTS - 2:        # keep slots on the native side: acquire returns
                self._submit_oldest()
            slot = self.w.acquire()
            dst = self.ring[slot].tensor[:m]
            if dev_src:
                _lib.memcpy_async(dst, flat[a:a + m], self.cs)
                ev = torch.cuda.Event()
                ev.record(self.cs)
            else:
                ctypes.memmove(dst.data_ptr(), flat[a:a + m].data_ptr(), m)
                ev = None
            self.pending.append((slot, ev, self.offs[file], m, file))
            self.offs[file] += m
            self.off += m

    def _submit_oldest(self):
        slot, ev, off, n, f = self.pending.popleft()
        if ev is not None:
            ev.synchronize()
        self.w.submit(slot, off, n, f)

    def close(self):
        if self.closed:
            return list(self.offs) if self.multi else self.off
        try:
            self._submit_done(block=True)
            if self.multi:
                self.w.finish_all(list(self.offs))
            else:
                self.w.finish(self.off)
        finally:
            self.closed = True
            _RING_LOCK.release()
        if self.stats is not None:
            self.stats.bytes += self.off
            self.stats.seconds += time.perf_counter() - self.t0
        return list(self.offs) if self.multi else self.off

    def abort(self):
        if self.closed:
            return
        try:
            for _, ev, _, _, _ in self.pending:
                if ev is not None:
                    ev.synchronize()
            self.pending.clear()
            self.w.abort()
        finally:
            self.closed = True
            _RING_LOCK.release()


def write_device(path: str, data: torch.Tensor, stats: WriteStats | None = None) -> int:
    """Write one device (or host) tensor's bytes to a new file at ``path``."""
    with PartWriter(path, data.device if isinstance(data, torch.Tensor) else None, stats) as w:
        w.write(data)
    return w.off


# A large partition may be written as several part files at once (context PartFileSplitBytes, at
# most SPLIT_MAX files): page-cache writes to one file serialise on its inode lock (~12 GB/s on the
# MI355X box), to distinct files they do not (40-93 GB/s, profiles/r4/filewrite_ab2.log).
SPLIT_MAX = 8


def write_device_pieces(paths: list, data: torch.Tensor, bounds: list, stats: WriteStats | None = None,
                        reuse: bool = False) -> list:
    """Write byte ranges [bounds[i], bounds[i + 1]) of ``data`` (a contiguous device or host tensor)
    to ``paths[i]``, every file at once: the chunks go out round-robin over the files, so the
    writer threads work on distinct inodes.  ``reuse``: files already at ``paths`` (recycled parts
    of a replaced table) are overwritten in place and cut to size, not truncated first.  Returns
    the file sizes."""
    from ..native import runtime
    from ..ops import _lib
    k = len(paths)
    assert len(bounds) == k + 1 and bounds[0] == 0
    flat = data.reshape(-1).view(torch.uint8)
    assert bounds[-1] <= flat.numel()
    t0 = time.perf_counter()
    ring = _ring()
    with _RING_LOCK:
        w = runtime().ChunkWriter(list(paths), [b.tensor.data_ptr() for b in ring], THREADS, reuse=reuse)
        dev_src = flat.is_cuda
        cs = None
        if dev_src:
            cs = torch.cuda.Stream(flat.device)
            cs.wait_stream(torch.cuda.current_stream(flat.device))
            flat.record_stream(cs)
        piece = min(CHUNK, ring[0].tensor.numel())
        pending = deque()
        done = False
        try:
            offs = [0] * k
            while any(bounds[i] + offs[i] < bounds[i + 1] for i in range(k)):
                for i in range(k):
                    a = bounds[i] + offs[i]
                    m = min(piece, bounds[i + 1] - a)
                    if m <= 0:
                        continue
                    while pending and (pending[0][1] is None or pending[0][1].query()):
                        slot, ev, f, off, n = pending.popleft()
                        w.submit(slot, off, n, f)
                    while len(pending) > SLOTS - 2:
                        slot, ev, f, off, n = pending.popleft()
                        if ev is not None:
                            ev.synchronize()
                        w.submit(slot, off, n, f)
                    slot = w.acquire()
                    dst = ring[slot].tensor[:m]
                    if dev_src:
                        _lib.memcpy_async(dst, flat[a:a + m], cs)
                        ev = torch.cuda.Event()
                        ev.record(cs)
                    else:
                        ctypes.memmove(dst.data_ptr(), flat[a:a + m].data_ptr(), m)
                        ev = None
                    pending.append((slot, ev, i, offs[i], m))
                    offs[i] += m
            while pending:
                slot, ev, f, off, n = pending.popleft()
                if ev is not None:
                    ev.synchronize()
                w.submit(slot, off, n, f)
            sizes = [bounds[i + 1] - bounds[i] for i in range(k)]
            w.finish_all(sizes)
            done = True
        finally:
            if not done:
                for _, ev, _, _, _ in pending:
                    if ev is not None:
                        ev.synchronize()
                w.abort()
    if stats is not None:
        stats.bytes += bounds[-1]
        stats.seconds += time.perf_counter() - t0
    return sizes

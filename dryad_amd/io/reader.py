"""File -> HBM: a part file read by the native ChunkReader (csrc/runtime/partreader.cpp: several
reader threads pread() 64 MB chunks into a ring of page-locked host buffers) while every ready
chunk is DMA'd to its place in the device buffer on a copy stream, so disk / page-cache reads,
PCIe transfers and the readers' next chunks overlap.  Replaces read -> bytes -> pageable H2D
(two host copies plus a bounce buffer).  Reference: the overlapped native channel reader,
DryadVertex/VertexHost/system/channel/src/channelbuffernativereader.cpp.
"""
from __future__ import annotations

import os
import threading
from collections import deque

import torch

CHUNK = 64 << 20
SLOTS = 8
THREADS = 8

_RING = None
_RING_LOCK = threading.Lock()


def _ring():
    """The process's pinned staging ring (registered once; reused by every read)."""
    global _RING
    with _RING_LOCK:
        if _RING is None:
            from ..ops._lib import PinnedHostBuffer
            _RING = [PinnedHostBuffer((CHUNK,)) for _ in range(SLOTS)]
        return _RING


class ReadStats:
    def __init__(self):
        self.bytes = 0
        self.seconds = 0.0
        self.chunks = 0


def _sized(ring) -> list:
    """The ring as (address, bytes) pairs: the native reader refuses a chunk larger than a buffer."""
    return [(b.tensor.data_ptr(), b.tensor.numel() * b.tensor.element_size()) for b in ring]


def read_to_device(path: str, device, offset: int = 0, length: int = -1, out: torch.Tensor | None = None,
                   stats: ReadStats | None = None) -> torch.Tensor:
    """Bytes [offset, offset + length) of ``path`` (to the end when length < 0) into a device
    uint8 tensor (``out`` when given).  Returns after the data is on the device (the copy stream
    is joined to the current stream)."""
    import time
    from ..native import runtime
    from ..ops import _lib
    t0 = time.perf_counter()
    size = os.path.getsize(path)
    length = max(0, size - offset) if length < 0 else min(length, max(0, size - offset))
    dev = torch.device(device)
    if out is None:
        out = torch.empty(length, dtype=torch.uint8, device=dev)
    out = out.view(-1)
    if out.numel() < length:
        raise ValueError("read_to_device: output buffer too small")
    if length == 0:
        return out[:0]
    ring = _ring()
    chunk = min(CHUNK, ring[0].tensor.numel())      # the ring may predate a CHUNK change
    with _RING_LOCK:           # one reader per process at a time owns the ring
        rd = runtime().ChunkReader(path, int(offset), int(length), chunk, _sized(ring), THREADS)
        cur = torch.cuda.current_stream(dev)
        cs = torch.cuda.Stream(dev)
        cs.wait_stream(cur)
        pending = deque()      # (slot, event) DMAs in flight
        try:
            while True:
                while pending and pending[0][1].query():
                    rd.release(pending.popleft()[0])
                if len(pending) == len(ring):      # every slot is in a DMA: wait for the oldest
                    s0, e0 = pending.popleft()
                    e0.synchronize()
                    rd.release(s0)
                got = rd.next(-1)
                if got is None:
                    break
                slot, ci, nb = got
                a = ci * chunk
                _lib.memcpy_async(out[a:a + nb], ring[slot].tensor[:nb], cs)
                ev = torch.cuda.Event()
                ev.record(cs)
                pending.append((slot, ev))
                if stats is not None:
                    stats.chunks += 1
            for s, e in pending:
                e.synchronize()
                rd.release(s)
            pending.clear()
        finally:
            for s, e in pending:
                e.synchronize()
            rd.stop()
        cur.wait_stream(cs)
    if stats is not None:
        stats.bytes += length
        stats.seconds += time.perf_counter() - t0
    return out[:length]


def read_rows_to_device(path: str, device, offset: int, n: int, stride: int, out: torch.Tensor,
                        stats: ReadStats | None = None) -> torch.Tensor:
    """``n`` fixed-width rows of ``stride`` bytes at ``offset`` of ``path`` into ``out``, an
    [n, stride] uint8 device view whose rows may sit at a wider pitch (e.g. the 128-byte-pitch
    sort input, ops/sort.sort_rows_pitch128).  A contiguous ``out`` is one read_to_device; a
    pitched one goes chunk by chunk (whole rows per chunk) through a device staging buffer and
    one strided copy per chunk, on the copy stream, behind the chunk's DMA."""
    import time
    from ..native import runtime
    from ..ops import _lib
    if out.shape[0] < n or out.shape[1] != stride:
        raise ValueError("read_rows_to_device: output view too small")
    if n == 0:
        return out[:0]
    if out[:n].is_contiguous():
        read_to_device(path, device, offset=offset, length=n * stride, out=out[:n].view(-1), stats=stats)
        return out[:n]
    t0 = time.perf_counter()
    dev = torch.device(device)
    length = n * stride
    if os.path.getsize(path) < offset + length:
        raise ValueError(f"read_rows_to_device: {path} holds fewer than {n} rows of {stride} bytes")
    ring = _ring()
    # whole rows per chunk, at most a ring buffer (the ring may predate a CHUNK change: a reader
    # told a chunk larger than its buffers would write past them)
    cb = (min(CHUNK, ring[0].tensor.numel()) // stride) * stride
    if cb == 0:
        raise ValueError(f"read_rows_to_device: {stride}-byte rows exceed the {ring[0].tensor.numel()}-byte ring buffers")
    stage = torch.empty(cb, dtype=torch.uint8, device=dev)
    with _RING_LOCK:
        rd = runtime().ChunkReader(path, int(offset), int(length), cb, _sized(ring), THREADS)
        cur = torch.cuda.current_stream(dev)
        cs = torch.cuda.Stream(dev)
        cs.wait_stream(cur)
        pending = deque()
        try:
            with torch.cuda.stream(cs):
                while True:
                    while pending and pending[0][1].query():
                        rd.release(pending.popleft()[0])
                    if len(pending) == len(ring):
                        s0, e0 = pending.popleft()
                        e0.synchronize()
                        rd.release(s0)
                    got = rd.next(-1)
                    if got is None:
                        break
                    slot, ci, nb = got
                    r0, nr = ci * (cb // stride), nb // stride
                    _lib.memcpy_async(stage[:nb], ring[slot].tensor[:nb], cs)
                    ev = torch.cuda.Event()
                    ev.record(cs)
                    pending.append((slot, ev))
                    out[r0:r0 + nr].copy_(stage[:nb].view(nr, stride))   # same stream: after the DMA,
                    if stats is not None:                                   # before the next one
                        stats.chunks += 1
            for s_, e_ in pending:
                e_.synchronize()
                rd.release(s_)
            pending.clear()
        finally:
            for s_, e_ in pending:
                e_.synchronize()
            rd.stop()
        cur.wait_stream(cs)
        stage.record_stream(cur)
    if stats is not None:
        stats.bytes += length
        stats.seconds += time.perf_counter() - t0
    return out[:n]


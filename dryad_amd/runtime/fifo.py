"""In-process FIFO channels and subgraph vertices (SURVEY C-5).

Reference: ``channelfifo.h:27-241`` / ``channelfifo.cpp`` (a bounded in-memory channel between
two vertices of one process) and ``DryadSubGraphVertex`` (``subgraphvertex.h:20-202``: several
vertex programs in one process joined by FIFOs, so a chain of stages streams records instead of
materialising every intermediate channel).

The queue is the native ``BlockFifo`` (``csrc/runtime/fifo.h``): blocks of records move between
threads without the GIL held while a side waits, the writer blocks once ``capacity_bytes`` are
queued (back pressure), ``close`` is end-of-stream, and a failure on either side aborts both
ends with the error text (the reference propagates an upstream vertex failure the same way).
"""
from __future__ import annotations

import pickle
import threading

from .. import native

OK, TIMEOUT, CLOSED, ABORTED = 0, 1, 2, 3


class FifoError(RuntimeError):
    """The other end of a FIFO channel failed (or the channel was used after close)."""


class FifoChannel:
    """A record channel over one native BlockFifo: ``write(records)`` on the producer thread,
    iteration on the consumer thread.  Records travel in blocks of ``batch`` records."""

    def __init__(self, capacity_bytes: int = 64 << 20, batch: int = 4096):
        self._f = native.runtime().BlockFifo(int(capacity_bytes))
        self.batch = max(1, int(batch))
        self.records_written = 0

    def _put(self, buf: list) -> bool:
        """False once the consumer has closed the channel (it needs no more records)."""
        st = self._f.put(pickle.dumps(buf, protocol=pickle.HIGHEST_PROTOCOL), -1)
        if st == ABORTED:
            raise FifoError(self._f.error())
        if st == CLOSED:
            return False
        self.records_written += len(buf)
        return True

    def write(self, records) -> int:
        """Write every record, then close (end of stream).  An exception in the producer aborts
        the channel so the consumer fails instead of seeing a short stream; a consumer that
        stopped early (``close``) ends the write quietly."""
        buf = []
        try:
            for r in records:
                buf.append(r)
                if len(buf) >= self.batch:
                    if not self._put(buf):
                        return self.records_written
                    buf = []
            if buf:
                self._put(buf)
        except BaseException as e:
            self.abort(f"{type(e).__name__}: {e}")
            raise
        self._f.close()
        return self.records_written

    def __iter__(self):
        while True:
            st, blk = self._f.get(-1)
            if st == OK:
                yield from pickle.loads(blk)
            elif st == CLOSED:
                return
            else:
                raise FifoError(self._f.error())

    def abort(self, why: str):
        self._f.abort(why)

    def close(self):
        """Consumer side: no more records wanted (an upstream writer stops at its next block)."""
        self._f.close()

    def stats(self) -> dict:
        return {"capacity": self._f.capacity(), "peak_bytes": self._f.peak_bytes(),
                "blocks": self._f.blocks_written(), "records": self.records_written}


def run_subgraph(source, vertices, capacity_bytes: int = 64 << 20, batch: int = 4096) -> list:
    """Run a chain of vertex bodies (each ``iterable -> iterable``) as one subgraph vertex: one
    thread per vertex, consecutive vertices joined by FIFO channels, the last one's output
    collected.  The first failure aborts every channel and is re-raised."""
    chans = [FifoChannel(capacity_bytes, batch) for _ in vertices]
    errors: list = []
    lock = threading.Lock()

    def fail(e):
        with lock:
            errors.append(e)
        for c in chans:
            c.abort(f"{type(e).__name__}: {e}")

    def body(i, fn):
        try:
            src = source if i == 0 else chans[i - 1]
            chans[i].write(fn(src))
            if i > 0:
                chans[i - 1].close()     # a vertex that stopped early releases its producer
        except BaseException as e:  # noqa: BLE001
            fail(e)

    threads = [threading.Thread(target=body, args=(i, fn), daemon=True, name=f"subgraph-v{i}")
               for i, fn in enumerate(vertices)]
    for t in threads:
        t.start()
    out = []
    try:
        out = list(chans[-1]) if chans else list(source)
    except FifoError as e:
        if not errors:
            errors.append(e)
    for t in threads:
        t.join()
    if errors:
        first = next((e for e in errors if not isinstance(e, FifoError)), errors[0])
        raise first
    return out

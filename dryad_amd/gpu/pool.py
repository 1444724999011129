"""HBM working-set pool of the GPU executor.

A 125 GB/GPU sort needs input rows + output rows + two entry arrays resident at once (~290 GB of
the 309 GB on an MI355X), so the executor cannot let each vertex allocate freely: large record
tables are carved out of one long-lived ``SortBuffers`` set that is reused job after job.  An HBM
output table (``hbm://``) pins the buffer set its rows live in until the table is deleted
(``ToStore(..., delete_if_exists=True)`` deletes at submission, like the reference's
CheckExistence(deleteIfExists) in DataProvider.cs:484-538).
"""
from __future__ import annotations

import threading

import torch

from ..ops import recordsort as RS


class BufferSet:
    def __init__(self, bufs: RS.SortBuffers, stride: int, layout: str = "plain"):
        self.bufs = bufs
        self.stride = stride
        # "plain": rows_in [cap, stride], rows_out [cap, stride], two E128 entry arrays.
        # "pitch128": rows_in [cap, 128] (records of `stride` <= 128 bytes, one aligned HBM line
        # each), rows_out [cap, stride], ent_a [cap] int64 compact entries, no ent_b (the radix
        # sort ping-pongs through rows_out: ops/sort.sort_rows_pitch128)
        self.layout = layout
        self.pins = 0
        self.in_use = False
        # set by a producer that also wrote rows_in's sort entries into bufs.ent_a:
        # (rows_in data_ptr, n, key_off, key_len, hi_range device tensor, entry format "e64" |
        # "e128"), or the format "gen" (no entries: a lazy gen://terasort read, see lazy_gen);
        # consumed by one sort
        self.keys_ready = None
        # (first record, seed): rows_in holds gen://terasort records first.. that were NOT written;
        # the distributed sort generates them straight into its send buckets, any other consumer
        # must call materialize() first
        self.lazy_gen = None

    def materialize(self, n: int):
        """Write the records a lazy gen://terasort read skipped (no-op otherwise)."""
        if self.lazy_gen is not None:
            from ..ops import terasort as TS
            first, seed = self.lazy_gen
            TS.generate(self.bufs.rows_in[:n], first, seed)
            self.lazy_gen = None
            if self.keys_ready is not None and self.keys_ready[5] == "gen":
                self.keys_ready = None

    def take_keys(self, rows, key_off: int, key_len: int):
        """(hi min, hi max, entry format) of the entries in ent_a for exactly these rows and key,
        or None.  One-shot: sorting reuses ent_a as scratch, so the claim is dropped either way."""
        kr, self.keys_ready = self.keys_ready, None
        if kr is None or rows is None:
            return None
        ptr_, n, off, ln, rng, fmt = kr
        if ptr_ != rows.data_ptr() or n != rows.shape[0] or off != key_off or ln != key_len:
            return None
        if rng is None:                  # "gen": no entries, the bounds are the whole key space
            return 0, (1 << 64) - 1, fmt
        mn, mx = (int(x) & ((1 << 64) - 1) for x in rng.cpu().tolist())
        return mn, mx, fmt

    @property
    def capacity(self):
        return self.bufs.capacity


# HBM kept free next to a sort working set: RCCL's own buffers are allocated at communicator
# creation (before this check runs), this covers the sampler, separators, kernel workspaces and
# the caching allocator's rounding
RESERVE_BYTES = 2 << 30


def working_set_bytes(capacity: int, stride: int, layout: str = "plain") -> int:
    cap = int(capacity) + 1024
    if layout == "pitch128":
        return cap * (128 + stride + 8)
    return cap * (2 * stride + 32)


def allocate(capacity: int, stride: int, device, layout: str = "plain") -> RS.SortBuffers:
    if layout == "plain":
        return RS.SortBuffers.allocate(capacity, stride, device)
    if layout != "pitch128" or stride > 128:
        raise ValueError(f"HbmPool: unknown layout {layout!r} for {stride}-byte rows")
    cap = int(capacity) + 1024
    # the output table is allocated before the 128-byte-pitch input (A/B: profiles/r3/alloc_order_ab.log)
    rows_out = torch.empty((cap, stride), dtype=torch.uint8, device=device)
    rows_in = torch.empty((cap, 128), dtype=torch.uint8, device=device)
    return RS.SortBuffers(rows_in=rows_in, rows_out=rows_out,
                          ent_a=torch.empty(cap, dtype=torch.int64, device=device),
                          ent_b=torch.empty(0, dtype=torch.int64, device=device))


def check_fits(capacity: int, stride: int, device, layout: str = "plain") -> None:
    """Refuse, with a clear error, an in-HBM sort working set (rows in + rows out + two entry
    arrays) that cannot fit this GPU; e.g. 1.25e9 TeraSort rows per GPU need 293 GB of the 309 GB.
    Larger partitions go through the out-of-core OrderBy (ops/extsort.py: ``ExternalSort=True``
    with a host:// or partfile:// output)."""
    if device.type != "cuda":
        return
    free, total = torch.cuda.mem_get_info(device)
    need = working_set_bytes(capacity, stride, layout)
    if need + RESERVE_BYTES > free:
        from ..errors import DryadLinqException, ErrorCode
        raise DryadLinqException(
            ErrorCode.FailedToAllocateNewNativeBuffer,
            f"in-HBM sort of {capacity} rows x {stride} B needs {need / 1e9:.1f} GB (+{RESERVE_BYTES / 1e9:.1f} GB "
            f"reserve) but only {free / 1e9:.1f} of {total / 1e9:.1f} GB HBM are free on {device}; use the "
            f"out-of-core OrderBy (ExternalSort=True, host:// or partfile:// output) or more GPUs")


class HbmPool:
    def __init__(self, device):
        self.device = device
        self.sets: list = []
        self.lock = threading.Lock()

    def acquire(self, capacity: int, stride: int, layout: str = "plain") -> BufferSet:
        with self.lock:
            for s in self.sets:
                if not s.in_use and s.pins == 0 and s.stride == stride and s.layout == layout \
                        and s.capacity >= capacity:
                    s.in_use = True
                    s.keys_ready = None
                    return s
            # drop idle sets before allocating a new one (HBM is the limit, not the allocator)
            keep = [s for s in self.sets if s.in_use or s.pins > 0]
            self.sets = keep
            torch.cuda.empty_cache() if self.device.type == "cuda" else None
            check_fits(capacity, stride, self.device, layout)
            s = BufferSet(allocate(capacity, stride, self.device, layout), stride, layout)
            s.in_use = True
            self.sets.append(s)
            return s

    def release(self, s: BufferSet):
        with self.lock:
            s.in_use = False

    def pin(self, s: BufferSet):
        with self.lock:
            s.pins += 1

    def unpin(self, s: BufferSet):
        with self.lock:
            s.pins = max(0, s.pins - 1)

    def clear(self):
        with self.lock:
            self.sets = [s for s in self.sets if s.in_use or s.pins > 0]

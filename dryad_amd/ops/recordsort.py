"""Distributed sort of fixed-width record tables resident in HBM (the OrderBy / RangePartition
vertex programs of the GPU executor).

The reference compiles ``OrderBy(keySel)`` into a sampling stage + ``RangePartition`` (CrossProduct
channels) + ``MergeSort``/``Sort`` (LinqToDryad/DryadLinqQueryGen.cs:2362-2474 CreateRangePartition,
:2476 VisitOrderBy; DryadLinqSampler.cs:38-246).  On one MI355X node this becomes, per rank:

  1. extract   — key bytes -> 16-byte (key, row) entries              [HIP: dr_extract_keys]
  2. sample    — deterministic per-rank sample (seeded by rank = vertex id, so idempotent under
                 re-execution), all-gather, sort, pick world-1 evenly spaced separators
  3. range-dest— per entry destination by binary search of the separators   [HIP: dr_range_dest_u128]
  4. partition — one stable counting pass on the destination byte            [HIP: dr_partition_pass_u128]
  5. pack      — gather rows into destination-contiguous send buffer        [HIP: dr_gather_rows]
  6. exchange  — count all-to-all + payload all-to-all-v over xGMI          [RCCL]
  7. local sort— extract + 80/96-bit LSD radix sort + row gather            [HIP]

With world size 1 steps 2-6 are skipped.  All buffers are preallocated by the caller so a step does
no HBM allocation (everything stays resident; 288 GB per GPU holds in + out + entries).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import torch

from ..parallel.comm import World, get_world
from ..parallel import shuffle
from . import sort as S
import os as _os

# local sort algorithm: "hybrid" (top-window LSD + in-LDS run sort, default), "prefix"
# (64-bit LSD + tie fix-up) or "lsd" (full-width LSD)
SORT_ALGO = _os.environ.get("DRYAD_SORT_ALGO", "hybrid")


def key_bits(key_len: int) -> tuple[int, int, int]:
    """(begin_bit, end_bit, lo_mask) of the composite E128 key for a key of key_len bytes."""
    assert 1 <= key_len <= 12
    if key_len <= 8:
        return 64 + 8 * (8 - key_len), 128, 0
    extra = key_len - 8
    begin = 64 - 8 * extra
    mask = ((1 << (8 * extra)) - 1) << begin
    return begin, 128, mask


@dataclass
class SortBuffers:
    """HBM working set for one rank's sort: rows in/out and two entry arrays."""
    rows_in: torch.Tensor
    rows_out: torch.Tensor
    ent_a: torch.Tensor
    ent_b: torch.Tensor

    @staticmethod
    def allocate(capacity: int, stride: int, device, slack: float = 0.0):
        cap = int(capacity * (1.0 + slack)) + 1024
        return SortBuffers(
            rows_in=torch.empty((cap, stride), dtype=torch.uint8, device=device),
            rows_out=torch.empty((cap, stride), dtype=torch.uint8, device=device),
            ent_a=torch.empty((cap, 2), dtype=torch.int64, device=device),
            ent_b=torch.empty((cap, 2), dtype=torch.int64, device=device),
        )

    @property
    def capacity(self) -> int:
        return self.rows_in.shape[0]


@dataclass
class SortStats:
    n_in: int = 0
    n_out: int = 0
    send_counts: list = field(default_factory=list)
    recv_counts: list = field(default_factory=list)


def local_sort_rows(rows: torch.Tensor, out: torch.Tensor, ent_a: torch.Tensor, ent_b: torch.Tensor,
                    key_off: int, key_len: int, descending: bool = False,
                    hi_bounds: tuple[int, int] | None = None, keys_ready: bool = False) -> torch.Tensor:
    """Sort fixed-width ``rows`` by their byte-string key into ``out`` (stable).

    ``hi_bounds`` = known (min, max) of the first 8 key bytes as a big-endian integer (e.g. this
    rank's range-partition bounds); lets the hybrid sort skip their common prefix without a pass.
    ``keys_ready``: ``ent_a[:n]`` already holds ``extract_keys(rows, key_off, key_len)`` (the
    producer emitted them, e.g. the fused TeraSort generator)."""
    n = rows.shape[0]
    if n == 0:
        return out[:0]
    e = ent_a[:n] if keys_ready else S.extract_keys(rows, key_off, key_len, 0, out=ent_a[:n])
    if descending:
        # invert the key bits (not the row index) so an ascending radix sort yields descending keys
        b0, _, lo_mask = key_bits(key_len)
        e[:, 1].bitwise_not_()
        if lo_mask:
            e[:, 0].bitwise_xor_(torch.tensor(lo_mask - (1 << 64) if lo_mask >= (1 << 63) else lo_mask,
                                              dtype=torch.int64, device=e.device))
    b0, b1, _ = key_bits(key_len)
    if SORT_ALGO == "hybrid":
        srt = S.sort_entries_hybrid(e, b0, b1, tmp=ent_b[:n], hi_bounds=None if descending else hi_bounds)
    elif SORT_ALGO == "prefix" and b0 < 64:
        srt = S.sort_entries_prefix(e, b0, tmp=ent_b[:n])
    else:
        srt = S.sort_entries(e, b0, b1, tmp=ent_b[:n])
    return S.gather_rows(rows, entries=srt, out=out[:n])


def choose_separators(entries: torch.Tensor, n: int, world: World, lo_mask: int, sample_target: int,
                      seed: int, tmp: torch.Tensor) -> torch.Tensor:
    """Sampler (reference DryadLinqSampler.cs:38-246): per-rank stride sample at ~0.001 (at least
    min(n, 16) keys, at most sample_target), all-gathered, sorted on the GPU, world-1 separators at
    evenly spaced ranks.  Deterministic given (rank, n, seed)."""
    m = max(1, min(n, max(16, min(sample_target, n // 1000 if n >= 16000 else n))))
    stride = max(1, n // m)
    off = (seed + world.rank * 7919) % stride if stride > 1 else 0
    samp = entries[off: off + stride * m: stride][:m].clone()
    # keep only key bits in lo
    samp[:, 0] = samp[:, 0] & _as_i64(lo_mask)
    allsamp = shuffle.all_gather_varlen(samp, world)
    total = allsamp.shape[0]
    scratch = torch.empty_like(allsamp)
    srt = S.sort_entries(allsamp.contiguous(), 0, 128, tmp=scratch)
    pos = torch.tensor([(j * total) // world.size for j in range(1, world.size)], dtype=torch.int64,
                       device=srt.device)
    return srt.index_select(0, pos).contiguous()


def rank_hi_bounds(seps: torch.Tensor, rank: int) -> tuple[int, int]:
    """(min, max) of key ``hi`` words that range partition ``rank`` can receive."""
    his = [int(x) & ((1 << 64) - 1) for x in seps[:, 1].tolist()]
    lo = his[rank - 1] if rank > 0 else 0
    hi = his[rank] if rank < len(his) else (1 << 64) - 1
    return lo, hi


def _as_i64(v: int) -> int:
    v &= (1 << 64) - 1
    return v - (1 << 64) if v >= (1 << 63) else v


def distributed_sort_rows(bufs: SortBuffers, n: int, key_off: int, key_len: int, world: World | None = None,
                          sample_target: int = 1 << 20, seed: int = 314159,
                          stats: SortStats | None = None, keys_ready: bool = False,
                          hi_bounds: tuple[int, int] | None = None) -> torch.Tensor:
    """Globally sort the first ``n`` rows of ``bufs.rows_in`` across all ranks.

    On return rank r holds, in ``bufs.rows_out[:n_r]``, the r-th key range in ascending order.
    ``bufs.rows_in`` is clobbered (it becomes the receive buffer).  ``keys_ready``: ``bufs.ent_a[:n]``
    already holds the rows' sort entries; ``hi_bounds``: known hi range of the local keys."""
    w = world or get_world()
    rows = bufs.rows_in[:n]
    if w.size == 1:
        out = local_sort_rows(rows, bufs.rows_out, bufs.ent_a, bufs.ent_b, key_off, key_len,
                              hi_bounds=hi_bounds, keys_ready=keys_ready)
        if stats is not None:
            stats.n_in = stats.n_out = n
        return out
    stride = rows.shape[1]
    b0, b1, lo_mask = key_bits(key_len)
    ent = bufs.ent_a[:n] if keys_ready else S.extract_keys(rows, key_off, key_len, 0, out=bufs.ent_a[:n])
    part_mask = lo_mask
    if key_len <= 10 and w.size < (1 << 16):
        # skew: equal keys must not all land on one rank.  Bits 47..32 of lo are free for keys of
        # <= 10 bytes; with the rank there (and the row index below it) every entry is unique, so
        # the sampled separators split runs of equal keys across ranks while the global order
        # (key, rank, row) stays a valid OrderBy order.
        ent[:, 0].bitwise_or_(w.rank << 32)
        part_mask = (1 << 64) - 1
    seps = choose_separators(ent, n, w, part_mask, sample_target, seed, bufs.ent_b)
    S.range_dest(ent, seps, part_mask)                                   # ent.hi := destination
    part, starts = S.partition_pass(ent, 64, out=bufs.ent_b[:n])        # stable by destination
    S.gather_rows(rows, entries=part, out=bufs.rows_out[:n])            # pack send buffer
    st = starts[: w.size + 1].cpu().tolist()
    send_counts = [st[i + 1] - st[i] for i in range(w.size)]
    recv_t = shuffle.exchange_counts(torch.tensor(send_counts, dtype=torch.int64), w)
    recv_counts = [int(x) for x in recv_t.tolist()]
    n_recv = sum(recv_counts)
    if n_recv > bufs.capacity:
        raise RuntimeError(f"range partition skew: rank {w.rank} receives {n_recv} rows > capacity {bufs.capacity}")
    send_flat = bufs.rows_out.view(-1)
    recv_flat = bufs.rows_in.view(-1)
    shuffle.alltoallv_bytes(send_flat, [c * stride for c in send_counts], recv_flat,
                            [c * stride for c in recv_counts], w)
    out = local_sort_rows(bufs.rows_in[:n_recv], bufs.rows_out, bufs.ent_a, bufs.ent_b, key_off, key_len,
                          hi_bounds=rank_hi_bounds(seps, w.rank))
    if stats is not None:
        stats.n_in, stats.n_out = n, n_recv
        stats.send_counts, stats.recv_counts = send_counts, recv_counts
    return out

"""Partitioned (grace) hash join of fixed-width row tables: HBM first, pinned host DRAM spill.

SURVEY §5.7: the reference scales data size by partitioning every stage and spilling to temp
files when RAM runs out (DryadLinqVertex.cs:9584-9615); its HashJoin vertex
(DryadLinqVertex.cs:852-897, ParallelHashJoin :6703-7315) builds a hash lookup of the
co-partitioned inner side and streams the outer side through it.  On a GPU node the memory tiers
are HBM (288 GB) -> pinned host DRAM (PCIe) and the join is a grace join:

  pass A (per table, streamed in chunks):
     W > 1: rows -> rank by hash(key) [HIP dr_grace_partition, contiguous send layout]
            -> RCCL all-to-all-v over xGMI
     rows -> bucket by hash(key) [HIP dr_grace_partition]: each bucket's rows land directly in
            its HBM bucket store (device fill counters, no host round trip), or — for the buckets
            that do not fit the HBM budget — in a staging area that a side stream copies to pinned
            host DRAM while the next chunk is partitioned
  pass B (per bucket pair): spilled buckets stream back to HBM on the side stream (one bucket
     ahead); build an open-addressing table over the build side's bucket (sized for the Infinity
     Cache), probe with the other side [HIP dr_ht_build / dr_ht_probe_*].

Buckets are sized by the build side (<= ~6M rows, a 134 MB table) and as many as fit the HBM
budget stay resident; only the remainder is spilled (hybrid hash join).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import torch

from . import _lib
from ._lib import c_i32, c_u32, c_u64, ptr, stream_of, vp
from ..parallel import shuffle
from ..parallel.comm import World
from . import relational as R
from . import sort as S

_lib.register_signatures({
    "dr_grace_workspace": (c_u64, [c_u64, c_u32, c_u32]),
    "dr_grace_partition": (c_i32, [vp, c_u64, c_u32, c_u32, c_u32, c_u64, c_i32, c_u32, vp, vp, vp, c_u32, vp, vp,
                                   vp, vp, c_u32, c_u32, c_i32, vp]),
    "dr_ht_build": (c_i32, [vp, c_u64, c_u32, c_u32, c_u32, c_u64, vp, c_i32, vp]),
    "dr_ht_probe_sum_workspace": (c_u64, []),
    "dr_ht_probe_sum": (c_i32, [vp, c_u64, c_u32, c_u32, c_u32, c_u64, vp, c_i32, vp, c_u32, c_u32, c_u32, vp, vp,
                                vp]),
    "dr_ht_probe_pairs": (c_i32, [vp, c_u64, c_u32, c_u32, c_u32, c_u64, vp, c_i32, vp, vp, vp, vp, c_i32, vp]),
})

_lib.register_signatures({
    "dr_radix_tile_rows": (c_u32, [c_u32]),
    "dr_radix_partition": (c_i32, [vp, vp, c_u32, c_u32, c_u32, c_u64, c_i32, c_i32, vp, vp, vp, c_u32, c_u64, c_u64,
                                   vp, vp, vp, vp]),
    "dr_radix_join_workspace": (c_u64, []),
    "dr_radix_join_sum": (c_i32, [vp, vp, vp, vp, vp, vp, c_u64, c_u32, c_u32, c_u32, c_u64, c_u32, c_u32, vp, vp, vp,
                                  vp, vp]),
})

HASH_SEED = 0x6A09E667F3BCC908
# radix join: two more digits of the same 64-bit key hash (the grace buckets use its low word)
# split every bucket into 2^13 partitions whose build side fits a 64 KiB LDS table
RADIX_PASSES = ((32, 7), (39, 6))
MAX_BUCKETS = 256
BUILD_ROWS_PER_BUCKET = 6_000_000     # table of 2^23 16-byte slots (134 MB) at load <= 0.72
SLACK = 1.02                          # per-bucket capacity over the even share


class Partitioner:
    """Device state of one partitioning target: nb destinations with row pointers, fill counters
    and capacities (device arrays), reused chunk after chunk."""

    def __init__(self, nb: int, device):
        self.nb = nb
        self.dev = device
        self.ptrs = torch.zeros(nb, dtype=torch.int64, device=device)
        self.fill = torch.zeros(nb, dtype=torch.int64, device=device)
        self.cap = torch.zeros(nb, dtype=torch.int64, device=device)
        self.counts = torch.zeros(nb, dtype=torch.int64, device=device)
        self.bases = torch.zeros(nb, dtype=torch.int64, device=device)
        self.overflow = torch.zeros(1, dtype=torch.int32, device=device)
        self._ws = None

    def workspace(self, n: int, stride: int) -> torch.Tensor:
        need = int(_lib.lib().dr_grace_workspace(c_u64(max(n, 1)), c_u32(stride), c_u32(self.nb)))
        if self._ws is None or self._ws.numel() < need:
            self._ws = torch.empty(need, dtype=torch.uint8, device=self.dev)
        return self._ws


def partition_rows(rows: torch.Tensor, key_off: int, key_len: int, part: Partitioner, shift: int = 0,
                   contig_from: int | None = None, seed: int = HASH_SEED, proj: tuple[int, int] | None = None,
                   unordered: bool = False):
    """Scatter ``rows`` [n, stride] uint8 by hash(key) into ``part``'s destinations.  Buckets below
    ``contig_from`` (default: all) append at their fill counters (bounded by cap, overflow flagged);
    buckets from ``contig_from`` on are laid out back to back from row 0 of their pointer.
    ``part.counts`` / ``part.bases`` receive this call's rows and first row per destination.
    ``proj = (byte offset, bytes)``: the destination rows are that slice of every row (column
    pruning in the same pass).  ``unordered``: rows of a destination may land in any order, so when
    every destination appends at its fill counter the count pass is skipped (one atomic
    reservation per tile and destination); ``part.counts`` / ``part.bases`` are then not written."""
    _lib.require_gpu_tensor(rows, "partition_rows")
    n, stride = rows.shape
    po, ow = proj if proj is not None else (0, stride)
    cf = part.nb if contig_from is None else contig_from
    ws = part.workspace(n, stride)
    _lib.call("dr_grace_partition", ptr(rows), c_u64(n), c_u32(stride), c_u32(key_off), c_u32(key_len),
              c_u64(seed & (2**64 - 1)), shift, c_u32(part.nb), ptr(part.ptrs), ptr(part.fill), ptr(part.cap),
              c_u32(cf), ptr(part.counts), ptr(part.bases), ptr(part.overflow), ptr(ws), c_u32(ow), c_u32(po),
              int(unordered), stream_of(rows))


def split_by_rank(rows: torch.Tensor, key_off: int, key_len: int, part: Partitioner, out: torch.Tensor,
                  proj: tuple[int, int] | None = None) -> list:
    """Rows (or their ``proj`` slice) grouped by destination rank (hash bits 32..63) into ``out``;
    returns per-rank counts."""
    part.ptrs.fill_(out.data_ptr())
    partition_rows(rows, key_off, key_len, part, shift=32, contig_from=0, proj=proj)
    return part.counts.tolist()


@dataclass
class SpillStats:
    radix_overflow: int = 0           # radix-join partitions joined through the global table
    spilled_bytes: int = 0
    buckets: int = 0
    resident: int = 0
    in_hbm: bool = False
    rows: dict = field(default_factory=dict)


class _TableStore:
    """One table's buckets: [0, resident) in one HBM tensor, the rest in pinned host DRAM."""

    def __init__(self, nb, cap_rows, stride, resident, device):
        self.nb, self.cap, self.stride, self.resident = nb, cap_rows, stride, resident
        self.hbm = torch.empty((max(resident, 0) * cap_rows, stride), dtype=torch.uint8, device=device)
        self.host = None
        if nb > resident:
            from ._lib import pinned_lease
            self.host = pinned_lease(((nb - resident) * cap_rows, stride))
        self.part = Partitioner(nb, device)
        base = self.hbm.data_ptr()
        rb = cap_rows * stride
        self._init_fill = torch.tensor([b * cap_rows for b in range(nb)], dtype=torch.int64)
        self.part.cap.copy_(torch.tensor([(b + 1) * cap_rows for b in range(nb)], dtype=torch.int64))
        self._hbm_base, self._rb = base, rb
        self.part.ptrs.fill_(base)
        self.host_fill = [0] * nb
        self.fill = None          # host copy of the final fills (rows per bucket) after pass A
        self.reset()

    def reset(self):
        self.part.fill.copy_(self._init_fill)
        self.part.overflow.zero_()
        self.host_fill = [0] * self.nb
        self.fill = None

    def set_staging(self, staging: torch.Tensor):
        ptrs = [self._hbm_base if b < self.resident else staging.data_ptr() for b in range(self.nb)]
        self.part.ptrs.copy_(torch.tensor(ptrs, dtype=torch.int64))

    def host_rows(self, b):
        k = b - self.resident
        return self.host.tensor[k * self.cap: k * self.cap + self.host_fill[b]]

    def finish(self):
        if int(self.part.overflow.item()):
            raise RuntimeError("grace join bucket overflow: a bucket received more than its capacity (skewed keys)")
        f = self.part.fill.tolist()
        self.fill = [f[b] - b * self.cap if b < self.resident else self.host_fill[b] for b in range(self.nb)]

    def hbm_rows(self, b):
        return self.hbm[b * self.cap: b * self.cap + self.fill[b]]

    def release(self):
        if self.host is not None:
            self.host.release()
            self.host = None
        self.hbm = None


class GraceHashJoin:
    """Grace join of two row tables produced chunk by chunk (``add_chunk(table, rows)``), then
    joined bucket by bucket (``buckets(build, probe)`` yields HBM row views).

    ``stride`` / ``key_off`` describe the input rows.  ``proj = (byte offset, bytes)`` prunes
    every row to the columns the join reads in the first partitioning pass (before the xGMI
    exchange, the bucket stores and any spill), so the stored rows are ``proj[1]`` bytes with the
    key at ``key_off - proj[0]``."""

    def __init__(self, world: World, stride: int, key_off: int, key_len: int, rows_per_rank: dict,
                 chunk_rows: int, hbm_budget: int | None = None, buckets: int | None = None,
                 build: str | None = None, proj: tuple[int, int] | None = None):
        if proj is not None and not (proj[0] <= key_off and key_off + key_len <= proj[0] + proj[1] <= stride):
            raise ValueError("grace join projection must keep the key bytes")
        self.proj = proj
        self.key_off_in = key_off
        if proj is not None:
            stride, key_off = proj[1], key_off - proj[0]
        self.w, self.stride, self.key_off, self.key_len = world, stride, key_off, key_len
        dev = world.device
        self.dev = dev
        W = world.size
        free = torch.cuda.mem_get_info(dev)[0]
        self.budget = int(hbm_budget if hbm_budget is not None else free * 0.92)
        names = list(rows_per_rank)
        self.build_name = build or names[0]
        nbuild = rows_per_rank[self.build_name]
        nb = buckets or max(1, min(MAX_BUCKETS, -(-nbuild // BUILD_ROWS_PER_BUCKET)))
        caps = {t: int(n / nb * SLACK) + 4096 for t, n in rows_per_rank.items()}
        pair = sum(caps.values()) * stride                     # one bucket of every table
        self.log_cap = max(4, math.ceil(math.log2(caps[self.build_name] / 0.7)))
        table_bytes = (1 << self.log_cap) * 16
        exch = (chunk_rows * stride + int(chunk_rows * 1.3 + 4096) * stride) if W > 1 else 0
        fixed = table_bytes + exch
        if pair * nb + fixed <= self.budget:
            resident = nb
        else:
            if buckets is None:
                nb = max(nb, 16)
                caps = {t: int(n / nb * SLACK) + 4096 for t, n in rows_per_rank.items()}
                pair = sum(caps.values()) * stride
                self.log_cap = max(4, math.ceil(math.log2(caps[self.build_name] / 0.7)))
                fixed = (1 << self.log_cap) * 16 + exch
            # spilled buckets need two staging areas (partitioning) and two stream-in pairs
            fixed += 2 * chunk_rows * stride + 2 * pair
            resident = max(0, min(nb, int((self.budget - fixed) // pair)))
        self.B, self.resident = nb, resident
        self.in_hbm = resident >= nb
        self.caps = caps
        self.stores = {t: _TableStore(nb, caps[t], stride, resident, dev) for t in rows_per_rank}
        self.stats = SpillStats(buckets=nb, resident=resident, in_hbm=self.in_hbm)
        self.table = torch.empty((1 << self.log_cap) * 2, dtype=torch.int64, device=dev)
        self.copy_stream = torch.cuda.Stream(dev)
        self.staging, self.staging_ev = [], []
        if not self.in_hbm:
            srows = int(chunk_rows * 1.3) + 4096 if W > 1 else chunk_rows
            self.staging = [torch.empty((srows, stride), dtype=torch.uint8, device=dev) for _ in range(2)]
            self.staging_ev = [None, None]
            self.stream_bufs = [{t: torch.empty((caps[t], stride), dtype=torch.uint8, device=dev)
                                 for t in rows_per_rank} for _ in range(2)]
        self._turn = 0
        self._scratch = None              # radix join: one store-sized buffer, allocated on first use
        if W > 1:
            self.rank_part = Partitioner(W, dev)
            self.sbuf = torch.empty((chunk_rows, stride), dtype=torch.uint8, device=dev)
            self.rbuf = torch.empty((int(chunk_rows * 1.3) + 4096, stride), dtype=torch.uint8, device=dev)

    def reset(self):
        for st in self.stores.values():
            st.reset()
        self.stats = SpillStats(buckets=self.B, resident=self.resident, in_hbm=self.in_hbm)

    # -------------------------------------------------------------- pass A
    def add_chunk(self, table: str, rows: torch.Tensor):
        W = self.w.size
        key_off, proj = self.key_off_in, self.proj
        if W > 1:
            send = split_by_rank(rows, key_off, self.key_len, self.rank_part, self.sbuf, proj)
            key_off, proj = self.key_off, None          # received rows are already pruned
            recv = shuffle.exchange_counts(torch.tensor(send, dtype=torch.int64), self.w).tolist()
            n_recv = sum(recv)
            if n_recv > self.rbuf.shape[0]:
                self.rbuf = torch.empty((int(n_recv * 1.2), self.stride), dtype=torch.uint8, device=self.dev)
            shuffle.alltoallv_bytes(self.sbuf.view(-1)[: sum(send) * self.stride], [c * self.stride for c in send],
                                    self.rbuf.view(-1)[: n_recv * self.stride], [c * self.stride for c in recv], self.w)
            rows = self.rbuf[:n_recv]
        st = self.stores[table]
        main = torch.cuda.current_stream(self.dev)
        if not self.in_hbm:
            k = self._turn
            self._turn ^= 1
            if self.staging_ev[k] is not None:
                main.wait_event(self.staging_ev[k])      # its previous chunk's spill copies are done
            if self.staging[k].shape[0] < rows.shape[0]:  # a received chunk can exceed chunk_rows
                self.staging[k] = torch.empty((int(rows.shape[0] * 1.2), self.stride), dtype=torch.uint8,
                                              device=self.dev)
            st.set_staging(self.staging[k])
        # a join does not need the input order inside a bucket: resident buckets fill without a count pass
        partition_rows(rows, key_off, self.key_len, st.part, shift=0, contig_from=st.resident, proj=proj,
                       unordered=True)
        if not self.in_hbm:
            counts = st.part.counts.tolist()          # one small D2H per chunk
            self.copy_stream.wait_stream(main)
            off = 0
            for b in range(st.resident, self.B):
                c = counts[b]
                if c:
                    if st.host_fill[b] + c > st.cap:
                        raise RuntimeError(f"grace join bucket {b} overflow ({st.host_fill[b] + c} > {st.cap} rows)")
                    kk = b - st.resident
                    dst = st.host.tensor[kk * st.cap + st.host_fill[b]: kk * st.cap + st.host_fill[b] + c]
                    _lib.memcpy_async(dst, self.staging[k][off: off + c], self.copy_stream)
                    st.host_fill[b] += c
                    self.stats.spilled_bytes += c * self.stride
                off += c
            ev = torch.cuda.Event()
            ev.record(self.copy_stream)
            self.staging_ev[k] = ev
        self.stats.rows[table] = self.stats.rows.get(table, 0) + rows.shape[0]

    def finish_partitioning(self):
        torch.cuda.current_stream(self.dev).wait_stream(self.copy_stream)
        for st in self.stores.values():
            st.finish()

    # -------------------------------------------------------------- pass B
    def buckets(self, build: str, probe: str):
        """Yield (b, build_rows_b, probe_rows_b) in HBM; spilled buckets stream in on the side
        stream one bucket ahead of the caller's work."""
        self.finish_partitioning()
        Bs, Ps = self.stores[build], self.stores[probe]
        main = torch.cuda.current_stream(self.dev)
        pending = None
        for b in range(self.B):
            if b < self.resident:
                yield b, Bs.hbm_rows(b), Ps.hbm_rows(b)
                continue
            cur = pending if pending is not None else self._stream_in(build, probe, b, 0)
            main.wait_stream(self.copy_stream)
            pending = self._stream_in(build, probe, b + 1, (b + 1 - self.resident) & 1) if b + 1 < self.B else None
            yield b, cur[0], cur[1]

    def _stream_in(self, build, probe, b, slot):
        main = torch.cuda.current_stream(self.dev)
        self.copy_stream.wait_stream(main)         # the slot's previous bucket has been consumed
        out = []
        for t in (build, probe):
            h = self.stores[t].host_rows(b)
            d = self.stream_bufs[slot][t][: h.shape[0]]
            _lib.memcpy_async(d, h, self.copy_stream)
            out.append(d)
        return out

    def join_sum_all(self, build: str, probe: str, col_b: int, col_p: int, acc: torch.Tensor) -> bool:
        """Every bucket pair at once through the LDS radix join (radix_join_sum) when all buckets
        are resident in HBM and the rows are narrow (pruned); False when the per-bucket path has
        to run instead."""
        if not self.in_hbm or self.stride != 16 or self.key_len > 8 or self.key_off % 4:   # dr_radix_join_sum
            return False
        self.finish_partitioning()
        Bs, Ps = self.stores[build], self.stores[probe]
        rows = max(Bs.hbm.shape[0], Ps.hbm.shape[0])
        if self._scratch is None or self._scratch.shape[0] < rows:
            free = torch.cuda.mem_get_info(self.dev)[0]
            if rows * self.stride > free * 0.9:
                return False
            self._scratch = torch.empty((rows, self.stride), dtype=torch.uint8, device=self.dev)
        segs = []
        for st in (Bs, Ps):
            segs.append((torch.arange(self.B, dtype=torch.int64, device=self.dev) * st.cap,
                         torch.tensor(st.fill, dtype=torch.int64, device=self.dev)))
        self.stats.radix_overflow = radix_join_sum(Bs.hbm, segs[0], Ps.hbm, segs[1], self.key_off, self.key_len,
                                                   col_b, col_p, acc, self._scratch)
        return True

    def join_sum_hybrid(self, build: str, probe: str, col_b: int, col_p: int, acc: torch.Tensor) -> bool:
        """The LDS radix join for a hybrid (partly spilled) join of 16-byte rows: the resident
        buckets all at once, then every spilled bucket pair as it streams back from host DRAM
        (the next pair's upload overlaps this pair's join).  False when the rows do not suit it."""
        if self.in_hbm or self.stride != 16 or self.key_len > 8 or self.key_off % 4:
            return False
        self.finish_partitioning()
        Bs, Ps = self.stores[build], self.stores[probe]
        cap = max(Bs.cap, Ps.cap)
        # scratch of the radix passes: a group of resident buckets at a time (whatever HBM is left)
        free = torch.cuda.mem_get_info(self.dev)[0] + (0 if self._scratch is None else self._scratch.numel())
        group = max(1, min(max(self.resident, 1), int(free * 0.8) // (cap * self.stride)))
        rows = group * cap
        if self._scratch is None or self._scratch.shape[0] < rows:
            self._scratch = None
            self._scratch = torch.empty((rows, self.stride), dtype=torch.uint8, device=self.dev)
        ovf = 0
        for g0 in range(0, self.resident, group):
            g1 = min(self.resident, g0 + group)
            segs = []
            for st in (Bs, Ps):
                segs.append((torch.arange(g1 - g0, dtype=torch.int64, device=self.dev) * st.cap,
                             torch.tensor(st.fill[g0:g1], dtype=torch.int64, device=self.dev)))
            ovf += radix_join_sum(Bs.hbm[g0 * Bs.cap: g1 * Bs.cap], segs[0], Ps.hbm[g0 * Ps.cap: g1 * Ps.cap],
                                  segs[1], self.key_off, self.key_len, col_b, col_p, acc, self._scratch)
        zero = torch.zeros(1, dtype=torch.int64, device=self.dev)
        for b, br, pr in self.buckets(build, probe):
            if b < self.resident or br.shape[0] == 0 or pr.shape[0] == 0:
                continue
            ovf += radix_join_sum(br, (zero, torch.tensor([br.shape[0]], dtype=torch.int64, device=self.dev)),
                                  pr, (zero, torch.tensor([pr.shape[0]], dtype=torch.int64, device=self.dev)),
                                  self.key_off, self.key_len, col_b, col_p, acc, self._scratch)
        self.stats.radix_overflow = ovf
        return True

    def clear_table(self):
        self.table.fill_(-1)

    def release(self):
        for st in self.stores.values():
            st.release()
        self._scratch = None


_RADIX_SCRATCH: dict = {}


def _counts_buf(n: int, dev) -> torch.Tensor:
    t = _RADIX_SCRATCH.get(("counts", dev))
    if t is None or t.numel() < n:
        t = _RADIX_SCRATCH[("counts", dev)] = torch.empty(max(n, 1 << 20), dtype=torch.int32, device=dev)
    return t


def radix_partition(rows: torch.Tensor, out: torch.Tensor, seg_begin: torch.Tensor, seg_len: torch.Tensor,
                    key_off: int, key_len: int, shift: int, bits: int, seed: int = HASH_SEED):
    """One stable radix-partition pass (dr_radix_partition): each segment [begin, begin + len) of
    ``rows`` is split by hash digit into ``out`` at the same rows.  Returns the new partitions'
    (start, len) device int64 tensors, segment-major (nseg * 2^bits)."""
    dev = rows.device
    rb = rows.shape[1]
    nseg = seg_begin.numel()
    T = int(_lib.lib().dr_radix_tile_rows(c_u32(rb)))
    tiles = (seg_len + (T - 1)) // T
    tile_base = torch.zeros(nseg + 1, dtype=torch.int64, device=dev)
    torch.cumsum(tiles, 0, out=tile_base[1:])
    ntiles = int(tile_base[-1].item())
    counts = _counts_buf(ntiles << bits, dev)
    ps = torch.empty(nseg << bits, dtype=torch.int64, device=dev)
    pl = torch.empty(nseg << bits, dtype=torch.int64, device=dev)
    _lib.call("dr_radix_partition", ptr(rows), ptr(out), c_u32(rb), c_u32(key_off), c_u32(key_len),
              c_u64(seed & (2**64 - 1)), shift, bits, ptr(seg_begin), ptr(seg_len), ptr(tile_base), c_u32(nseg),
              c_u64(ntiles), c_u64(rows.shape[0]), ptr(counts), ptr(ps), ptr(pl), stream_of(rows))
    return ps, pl


def radix_join_sum(brows: torch.Tensor, bseg, prows: torch.Tensor, pseg, key_off: int, key_len: int, col_b: int,
                   col_p: int, acc: torch.Tensor, scratch: torch.Tensor, seed: int = HASH_SEED):
    """``join_sum`` of every aligned segment pair at once: both sides radix-partitioned further
    (RADIX_PASSES, through ``scratch`` and back, so ``brows`` / ``prows`` are reordered within
    their segments) into partitions joined in LDS (dr_radix_join_sum).  Partitions too large for
    the LDS table (key skew) go through the global hash table.  ``bseg`` / ``pseg`` = (begin, len)
    device int64 tensors of the segments (e.g. the grace buckets)."""
    dev = brows.device
    parts = []
    for rows, (sb, sl) in ((brows, bseg), (prows, pseg)):
        tmp = scratch[: rows.shape[0]]
        (s1, b1), (s2, b2) = RADIX_PASSES
        ps, pl = radix_partition(rows, tmp, sb, sl, key_off, key_len, s1, b1, seed)
        ps, pl = radix_partition(tmp, rows, ps, pl, key_off, key_len, s2, b2, seed)
        parts.append((ps, pl))
    (bs, bl), (ps, pl) = parts
    nparts = bs.numel()
    ovf_count = torch.zeros(1, dtype=torch.int32, device=dev)
    ovf_list = torch.empty(nparts, dtype=torch.int32, device=dev)
    ws = _RADIX_SCRATCH.get(("ws", dev))
    if ws is None:
        ws = _RADIX_SCRATCH[("ws", dev)] = torch.empty(int(_lib.lib().dr_radix_join_workspace()), dtype=torch.uint8,
                                                       device=dev)
    _lib.call("dr_radix_join_sum", ptr(brows), ptr(bs), ptr(bl), ptr(prows), ptr(ps), ptr(pl), c_u64(nparts),
              c_u32(brows.shape[1]), c_u32(key_off), c_u32(key_len), c_u64(seed & (2**64 - 1)), c_u32(col_b),
              c_u32(col_p), ptr(ovf_count), ptr(ovf_list), ptr(acc), ptr(ws), stream_of(brows))
    n_ovf = int(ovf_count.item())
    if n_ovf:
        for p in sorted(ovf_list[:n_ovf].tolist()):
            b0, nb_, p0, np_ = (int(x) for x in (bs[p], bl[p], ps[p], pl[p]))
            lc = ht_log_cap(nb_)
            table = torch.empty((1 << lc) * 2, dtype=torch.int64, device=dev)
            join_sum(brows[b0:b0 + nb_], prows[p0:p0 + np_], key_off, key_len, col_b, col_p, acc, table, lc, seed)
    return n_ovf


def ht_log_cap(n_build: int) -> int:
    return max(4, math.ceil(math.log2(max(n_build, 1) / 0.7)))


def join_sum(build_rows: torch.Tensor, probe_rows: torch.Tensor, key_off: int, key_len: int, col_build: int,
             col_probe: int, acc: torch.Tensor, table: torch.Tensor, log_cap: int, seed: int = HASH_SEED):
    """acc (int64[3]) += (matches, sum of probe int64 column at byte col_probe over matches, sum of
    the matched build rows' int64 column at byte col_build): the decomposable aggregate of a join
    whose result selector is linear in one column per side, fused into the probe."""
    nb, sb = build_rows.shape
    npr, sp = probe_rows.shape
    assert nb * 10 <= 9 * (1 << log_cap) and table.numel() * 8 >= (1 << log_cap) * 16
    table[: (1 << log_cap) * 2].fill_(-1)
    s = stream_of(probe_rows)
    ws = _probe_ws(probe_rows.device)
    _lib.call("dr_ht_build", ptr(build_rows), c_u64(nb), c_u32(sb), c_u32(key_off), c_u32(key_len),
              c_u64(seed & (2**64 - 1)), ptr(table), log_cap, s)
    _lib.call("dr_ht_probe_sum", ptr(probe_rows), c_u64(npr), c_u32(sp), c_u32(key_off), c_u32(key_len),
              c_u64(seed & (2**64 - 1)), ptr(table), log_cap, ptr(build_rows), c_u32(sb), c_u32(col_probe),
              c_u32(col_build), ptr(acc), ptr(ws), s)
    return acc


_PROBE_WS = {}


def _probe_ws(dev):
    t = _PROBE_WS.get(dev)
    if t is None:
        t = _PROBE_WS[dev] = torch.empty(int(_lib.lib().dr_ht_probe_sum_workspace()), dtype=torch.uint8, device=dev)
    return t


def hash_join_pairs(build_rows: torch.Tensor, probe_rows: torch.Tensor, key_off: int, key_len: int,
                    seed: int = HASH_SEED):
    """(probe row, build row) index pairs of equal keys, grouped by probe row in probe order."""
    nb, sb = build_rows.shape
    npr, sp = probe_rows.shape
    dev = probe_rows.device
    if nb == 0 or npr == 0:
        z = torch.empty(0, dtype=torch.int64, device=dev)
        return z, z
    lc = ht_log_cap(nb)
    table = torch.full(((1 << lc) * 2,), -1, dtype=torch.int64, device=dev)
    s = stream_of(probe_rows)
    sd = c_u64(seed & (2**64 - 1))
    _lib.call("dr_ht_build", ptr(build_rows), c_u64(nb), c_u32(sb), c_u32(key_off), c_u32(key_len), sd, ptr(table),
              lc, s)
    count = torch.empty(npr, dtype=torch.int64, device=dev)
    _lib.call("dr_ht_probe_pairs", ptr(probe_rows), c_u64(npr), c_u32(sp), c_u32(key_off), c_u32(key_len), sd,
              ptr(table), lc, ptr(count), ptr(None), ptr(None), ptr(None), 0, s)
    offs = R.scan_exclusive(count)
    total = int((offs[-1] + count[-1]).item())
    po = torch.empty(total, dtype=torch.int64, device=dev)
    bo = torch.empty(total, dtype=torch.int64, device=dev)
    _lib.call("dr_ht_probe_pairs", ptr(probe_rows), c_u64(npr), c_u32(sp), c_u32(key_off), c_u32(key_len), sd,
              ptr(table), lc, ptr(count), ptr(offs), ptr(po), ptr(bo), 1, s)
    return po, bo


def sort_merge_join_pairs(left: torch.Tensor, right: torch.Tensor, key_off: int, key_len: int):
    """Row-index pairs (l, r) with equal key bytes (radix sort both sides + merge ranges)."""
    if left.shape[0] == 0 or right.shape[0] == 0:
        z = torch.empty(0, dtype=torch.int64, device=left.device)
        return z, z
    b0, _, lo_mask = _bits(key_len)
    el = S.sort_entries_hybrid(S.extract_keys(left, key_off, key_len, 0), b0)
    er = S.sort_entries_hybrid(S.extract_keys(right, key_off, key_len, 0), b0)
    oo, ii, _ = R.merge_join_pairs(el, er, lo_mask)
    return oo, ii


def _bits(key_len):
    from .recordsort import key_bits
    return key_bits(key_len)

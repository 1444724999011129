"""Out-of-core distributed sort of fixed-width row tables: HBM -> pinned host DRAM spill.

The in-HBM OrderBy (ops/recordsort.distributed_sort_rows) needs input rows + output rows + entry
arrays resident at once, ~2.3x the data.  A partition larger than that (the 1- and 2-GPU points of
a 1 TB TeraSort) is sorted here in range buckets that each fit the HBM budget.  The
reference does the same job on the CPU with sorted 2M-element runs spilled to temp files and a
<=16-way merge (``ParallelSort`` + ``FileEnumerable``, LinqToDryad/DryadLinqVertex.cs:9366-9367,
9584-9615, 10733); on MI355X a *sample-partition* external sort is cheaper than a merge: every row
crosses PCIe exactly twice in each direction and each bucket is one in-HBM radix sort.

Per rank (one process per GPU, W ranks):

  0. sample    — deterministic strided sample of the local rows (host sources: read straight out of
                 host memory; generator sources: one generate pass), all-gathered and sorted on the
                 GPU; W*P-1 separators cut the key space into P buckets per rank, each sized to ~70%
                 of what one in-HBM sort can hold                                   [HIP + RCCL]
  1. count     — stream the input chunk by chunk (host -> HBM DMA or the fused generator): extract
                 the key entries, range destination, histogram per (chunk, bucket); all-gathered, so
                 every rank knows every piece's size and final host offset up front      [HIP]
  2. partition — stream the input again: LDS-staged bucket scatter of whole rows
                 (dr_bucket_scatter_rows); W > 1: one all-to-all-v per chunk over xGMI; the bucket
                 pieces go straight to their final host region by DMA on a copy stream that runs
                 under the next chunk's kernels                                  [HIP + RCCL + DMA]
  3. sort      — per bucket: host -> HBM, hybrid/compact radix sort + row gather, HBM -> host in
                 place; the next bucket's upload and the previous bucket's download overlap the
                 sort (two copy streams, both PCIe directions busy)                     [HIP + DMA]

Hybrid (``resident=True``): the phases work in a fraction of the HBM budget (smaller chunks and
buckets) and the rest holds whole range buckets: after the count pass the largest suffix of this
rank's buckets that fits stays in HBM -- their pieces are copied device to device in the partition
pass, sorted in place in the sort pass, and returned in HBM (a ``TieredRows`` table: host buckets
first, then the resident ones).  Only the overflow crosses PCIe: 2(1 - f) bytes per input byte for
a resident fraction f instead of 3.

Equal keys are split across buckets (and ranks) by a (rank, chunk, row) tie tag in the spare entry
bits, so skewed keys still fit; the order is then the source order (rank 0's rows first, each rank
in row order), i.e. the sort is stable.  With
``keep_ties`` the rank boundaries keep every run of equal keys on one rank (the planner's
partitioned-by-key guarantee, DataSetInfo), only the buckets inside a rank split them.
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass, field

import torch

from ..io.hosttable import HostRows, TieredRows, is_registered
from ..parallel import shuffle
from ..parallel.comm import World, get_world
from . import _lib
from . import recordsort as RS
from . import sort as S

_M64 = (1 << 64) - 1
FILL_TARGET = 0.7            # planned bucket size as a fraction of one in-HBM sort's capacity
COPY_PIECE = 512 << 20       # bytes per DMA piece of a host <-> HBM copy


def _i64(v: int) -> int:
    v &= _M64
    return v - (1 << 64) if v >= (1 << 63) else v


@dataclass
class ExtSortStats:
    n_in: int = 0
    n_out: int = 0
    chunks: int = 0
    chunk_rows: int = 0
    buckets: int = 0
    bucket_cap: int = 0
    max_bucket: int = 0
    bytes_h2d: int = 0
    bytes_d2h: int = 0
    tier: str = "dram"           # where the output rows live: "dram" (pinned) or "disk" (mapped file)
    resident_rows: int = 0       # hybrid: rows of the buckets kept (sorted) in HBM
    resident_buckets: int = 0
    seconds: dict = field(default_factory=dict)


# ------------------------------------------------------------------------------------------------
# chunked sources
class ChunkSource:
    """A partition read chunk by chunk into HBM.  ``fill(lo, hi, out, copy_stream)`` writes rows
    [lo, hi) into ``out`` (device rows) and returns the stream the data is ready on
    (``None`` = the current stream)."""
    n: int = 0
    stride: int = 0
    dma = False          # fill is a host -> device copy (counts toward bytes_h2d)

    def fill(self, lo: int, hi: int, out: torch.Tensor, copy_stream):
        raise NotImplementedError

    def sample_rows(self, idx: torch.Tensor, scratch: torch.Tensor, chunk_rows: int) -> torch.Tensor:
        """Device rows at the sorted local indices ``idx`` (int64, host).  Default: stream every
        chunk that holds a sampled row through ``scratch`` and pick the rows on the device."""
        dev = scratch.device
        parts = []
        for c0 in range(0, self.n, chunk_rows):
            c1 = min(self.n, c0 + chunk_rows)
            sel = idx[(idx >= c0) & (idx < c1)]
            if sel.numel() == 0:
                continue
            st = self.fill(c0, c1, scratch[: c1 - c0], None)
            if st is not None:
                torch.cuda.current_stream(dev).wait_stream(st)
            parts.append(scratch.index_select(0, (sel - c0).to(dev)))
        if not parts:
            return torch.empty((0, self.stride), dtype=torch.uint8, device=dev)
        return torch.cat(parts)


class GenTeraSortSource(ChunkSource):
    """``gen://terasort`` rows [first, first + n) produced by the HIP generator in place."""

    def __init__(self, first: int, n: int, seed: int):
        from . import terasort as TS
        self.TS = TS
        self.first, self.n, self.seed, self.stride = first, n, seed, TS.RECORD_BYTES

    def fill(self, lo, hi, out, copy_stream):
        self.TS.generate(out[: hi - lo], self.first + lo, self.seed)
        return None


class HostRowsSource(ChunkSource):
    """A ``HostRows`` table (pinned host memory): chunks arrive by DMA on the copy stream."""
    dma = True

    def __init__(self, rows: HostRows):
        self.rows, self.n, self.stride = rows, rows.n, rows.stride
        self.key_spec = (rows.key_off, rows.key_len)

    def fill(self, lo, hi, out, copy_stream):
        _copy(out[: hi - lo], self.rows.rows[lo:hi], copy_stream)
        return copy_stream

    def sample_rows(self, idx, scratch, chunk_rows):
        return self.rows.rows.index_select(0, idx).to(scratch.device)


class MappedRowsSource(ChunkSource):
    """Raw fixed-width rows of a partfile part (``format: rows``), memory-mapped: each chunk is
    copied from the page cache / disk into a pinned staging buffer, then DMA'd to HBM."""
    dma = True

    def __init__(self, mm, key_off: int = 0, key_len: int | None = None):
        self.mm, self.n, self.stride = mm, mm.shape[0], mm.shape[1]
        self.key_spec = (key_off, key_len or self.stride)
        self._stage = None
        self._last = None                      # stream of the last DMA out of the staging buffer

    def fill(self, lo, hi, out, copy_stream):
        if self._last is not None:
            self._last.synchronize()           # the previous chunk has left the staging buffer
        if self._stage is None or self._stage.n < hi - lo:
            if self._stage is not None:
                self._stage.release()
            self._stage = HostRows(hi - lo, self.stride)
        self._stage.rows[: hi - lo].numpy()[:] = self.mm[lo:hi]
        st = copy_stream if copy_stream is not None else torch.cuda.current_stream(out.device)
        _copy(out[: hi - lo], self._stage.rows[: hi - lo], st)
        self._last = st
        return copy_stream

    def sample_rows(self, idx, scratch, chunk_rows):
        import numpy as np
        return torch.from_numpy(np.ascontiguousarray(self.mm[idx.numpy()])).to(scratch.device)


def _copy(dst: torch.Tensor, src: torch.Tensor, stream):
    """DMA between a device tensor and a host tensor on ``stream`` (page-locked host memory goes
    through hipMemcpyAsync directly; anything else through torch)."""
    host = src if dst.is_cuda else dst
    if stream is None:
        stream = torch.cuda.current_stream(dst.device if dst.is_cuda else src.device)
    if host.numel() == 0:
        return
    if is_registered(host) or host.is_pinned():
        # multi-GB copies go as <= 512 MB pieces: one huge DMA in one direction was measured not
        # to overlap the other direction's (27 vs 47 GB/s per direction with 11 GB buckets)
        rows = dst.shape[0]
        per = max(1, COPY_PIECE // max(1, dst[:1].numel() * dst.element_size())) if dst.dim() > 1 else COPY_PIECE
        if rows <= per:
            _lib.memcpy_async(dst, src, stream)
        else:
            for a in range(0, rows, per):
                _lib.memcpy_async(dst[a:a + per], src[a:a + per], stream)
    else:
        with torch.cuda.stream(stream):
            dst.copy_(src, non_blocking=False)


class _Arena:
    """One HBM allocation carved into the phase's working buffers (phases reuse the same bytes, so
    the caching allocator never holds two phases' layouts at once)."""

    def __init__(self, nbytes: int, device):
        self.buf = torch.empty(max(nbytes, 256), dtype=torch.uint8, device=device)
        self.off = 0

    def reset(self):
        self.off = 0

    def take(self, shape, dtype=torch.uint8) -> torch.Tensor:
        esz = torch.empty(0, dtype=dtype).element_size()
        nb = esz * math.prod(shape)
        a = (self.off + 255) & ~255
        if a + nb > self.buf.numel():
            raise MemoryError("extsort arena overflow")
        self.off = a + nb
        return self.buf[a:a + nb].view(dtype).view(*shape)


def default_budget(device) -> int:
    free, _ = torch.cuda.mem_get_info(device)
    return int(free * 0.8)


def plan_geometry(n_rank_max: int, n_total: int, stride: int, W: int, budget: int):
    """(chunk_rows, bucket_cap, buckets per rank) for a budget of ``budget`` HBM bytes."""
    usable = max(budget - (1 << 16), 1 << 16)             # alignment padding of the carved buffers
    crow = 4 * stride + 16 + (3 * stride if W > 1 else 0)
    chunk_rows = max(1, min(usable // crow, (1 << 31) - 1, max(n_rank_max, 1)))
    bucket_cap = max(2, usable // (4 * stride + 32))
    per_rank = -(-n_total // W)
    P = max(1, math.ceil(per_rank / (FILL_TARGET * bucket_cap)))
    if W * P > 256:
        raise RuntimeError(f"external sort: {n_total} rows of {stride} B need {W * P} range buckets with "
                           f"a {budget / 1e9:.1f} GB HBM budget (at most 256); raise the budget")
    return chunk_rows, bucket_cap, P


def _separators(srt: torch.Tensor, W: int, P: int, tie_bits: bool, lo_key_mask: int, part_mask: int):
    """W*P-1 ascending separators from the sorted sample: W-1 rank boundaries at even sample
    quantiles, then P-1 bucket boundaries at even quantiles of each rank's own share of the sample
    (so a rank that keeps a long run of equal keys still gets evenly filled buckets).
    ``tie_bits``: the rank boundaries take every tuple of their key (tie tag all ones)."""
    dev, T = srt.device, srt.shape[0]
    none = torch.zeros((0, 2), dtype=torch.int64, device=dev)
    rsep = srt.index_select(0, torch.tensor([(r * T) // W for r in range(1, W)], dtype=torch.int64,
                                            device=dev)).clone() if W > 1 else none
    if tie_bits and W > 1:
        rsep[:, 0] |= _i64(_M64 & ~lo_key_mask)
    # each sample's rank = #rank separators strictly below it (the kernel's own comparison)
    bounds = [0] * (W + 1)
    bounds[W] = T
    if W > 1:
        d = S.range_dest(srt.clone(), rsep, part_mask)[:, 1]
        cnt = torch.bincount(d, minlength=W).tolist()
        for r in range(W):
            bounds[r + 1] = bounds[r] + cnt[r]
    parts = []
    for r in range(W):
        a, b = bounds[r], bounds[r + 1]
        if P > 1 and b > a:
            idx = [a + (j * (b - a)) // P for j in range(1, P)]
            parts.append(srt.index_select(0, torch.tensor(idx, dtype=torch.int64, device=dev)))
        elif P > 1:       # no sample in this rank's range: its buckets are empty
            fill = rsep[r:r + 1] if r < W - 1 else (rsep[r - 1:r] if r > 0 else srt[T - 1:T])
            parts.append(fill.expand(P - 1, 2))
        if r < W - 1:
            parts.append(rsep[r:r + 1])
    return torch.cat(parts).contiguous() if parts else none


HYBRID_WORK_FRACTION = None    # fixed share of the budget for the phases' buffers (None: sized)
HYBRID_MIN_WORK = 2 << 30
HYBRID_BUCKETS = 72            # target range buckets per rank in hybrid mode


def hybrid_work(budget: int, rank_bytes: int, fraction: float | None = HYBRID_WORK_FRACTION) -> int:
    """HBM for the phases' buffers in hybrid mode (the rest holds resident buckets).  Sized so a
    rank gets about HYBRID_BUCKETS range buckets: fewer, larger buckets would leave less room for
    resident ones; many more make the partition pass's per-(chunk, bucket) host copies too small
    (measured: 108 buckets x 73 chunks halved the download rate, 72 x 49 kept it at 52 GB/s)."""
    if fraction is not None:
        w = int(budget * fraction)
    else:
        # bucket = FILL_TARGET * cap rows, cap = work / (4 stride + 32) ~ work / (4.32 stride)
        w = int(rank_bytes * 4.32 / (FILL_TARGET * HYBRID_BUCKETS))
    return min(budget, max(w, min(HYBRID_MIN_WORK, budget // 2)), max(budget // 2, 1))


def external_sort(src: ChunkSource, key_off: int, key_len: int, world: World | None = None,
                  budget: int | None = None, keep_ties: bool = False, sample_target: int = 1 << 20,
                  seed: int = 314159, stats: ExtSortStats | None = None,
                  out: HostRows | None = None, out_factory=None, resident: bool = False,
                  work_fraction: float = HYBRID_WORK_FRACTION, descending: bool = False):
    """Globally sort the rows of ``src`` (this rank's partition) by the byte-string key
    [key_off, key_off + key_len) (memcmp order, key_len <= 12).  Rank r returns the r-th key range
    as a ``HostRows`` table in pinned host memory.  ``budget``: HBM bytes the sort may use
    (default 80% of free HBM).  ``out``: a preallocated host table to write into when it is large
    enough (the result is then a view of its first rows); ``out_factory(n_out)``: builds the
    output table once this rank's row count is known (e.g. a memory-mapped part file,
    ``HostRows.mapped``, for outputs larger than host memory).  ``resident``: hybrid mode (module
    docstring); returns a ``TieredRows`` table when some buckets stayed in HBM.  ``descending``
    (OrderByDescending, the reference's ParallelSort with isDescending, DryadLinqVertex.cs:
    9330-9335): the key bits of every entry are inverted (recordsort.invert_keys) before sampling,
    range destination and each bucket's sort, so rank 0 / bucket 0 hold the largest keys; the tie
    tags are not inverted, so equal keys keep the source order (a stable descending sort)."""
    w = world or get_world()
    W, me = w.size, w.rank
    dev = w.device if w.device.type == "cuda" else torch.device("cuda", torch.cuda.current_device())
    stats = stats if stats is not None else ExtSortStats()
    stride, n = src.stride, src.n
    if not 1 <= key_len <= 12 or key_off + key_len > stride:
        raise ValueError("external_sort: key must be 1..12 bytes inside the row")
    t_all = time.perf_counter()
    budget = int(budget or default_budget(dev))
    tot = torch.tensor([n, n], dtype=torch.int64, device=dev if w.backend == "nccl" else "cpu")
    nmax = tot[:1].clone()
    shuffle.all_reduce_(tot[:1], "sum", w)
    shuffle.all_reduce_(nmax, "max", w)
    n_total, n_rank_max = int(tot[0]), int(nmax[0])
    work = hybrid_work(budget, -(-n_total // W) * stride, work_fraction) if resident else budget
    chunk_rows, bucket_cap, P = plan_geometry(n_rank_max, n_total, stride, W, work)
    C = max(1, -(-n_rank_max // chunk_rows))
    C_local = -(-n // chunk_rows)
    _, _, lo_key_mask = RS.key_bits(key_len)
    split = key_len <= 10 and C * W < (1 << 16)
    part_mask = _M64 if split else lo_key_mask
    stats.n_in, stats.chunks, stats.chunk_rows, stats.buckets, stats.bucket_cap = n, C, chunk_rows, P, bucket_cap
    arena = _Arena(work, dev)
    comp = torch.cuda.current_stream(dev)
    h2d, d2h = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    tag_of = lambda c: ((me * C + c) << 32)  # noqa: E731  (rank-major: the global source order)

    # ---------------------------------------------------------------- 0. sample + separators
    t0 = time.perf_counter()
    G = W * P
    m = min(n, max(256 * G, min(sample_target, max(n // 1000, 16))))
    seps, srows = None, None
    arena.reset()
    scratch = arena.take((chunk_rows, stride))
    ent = arena.take((chunk_rows, 2), torch.int64)
    if m > 0:
        stride_s = max(1, n // m)
        off = (seed + me * 7919) % stride_s if stride_s > 1 else 0
        idx = torch.arange(off, n, stride_s, dtype=torch.int64)[:m]
        srows = src.sample_rows(idx, scratch, chunk_rows)
        samp = S.extract_keys(srows.contiguous(), key_off, key_len, 0)
        if descending:
            RS.invert_keys(samp, key_len)
        if split:
            c_idx = idx // chunk_rows
            tag = ((me * C + c_idx) << 32) | (idx - c_idx * chunk_rows)
            samp[:, 0] = (samp[:, 0] & _i64(lo_key_mask)) | tag.to(dev)
        samp[:, 0] &= _i64(part_mask)
    else:
        samp = torch.empty((0, 2), dtype=torch.int64, device=dev)
    allsamp = shuffle.all_gather_varlen(samp, w)
    if allsamp.shape[0] == 0:
        allsamp = torch.zeros((1, 2), dtype=torch.int64, device=dev)
    srt = S.sort_entries(allsamp.contiguous(), 0, 128, tmp=torch.empty_like(allsamp))
    seps = _separators(srt, W, P, keep_ties and split, lo_key_mask, part_mask)
    seps_hi = [int(x) & _M64 for x in seps[:, 1].tolist()]
    del srows, samp, allsamp, srt
    stats.seconds["sample"] = time.perf_counter() - t0

    def entries(c, rows_c, out_e):
        e = S.extract_keys(rows_c, key_off, key_len, 0, out=out_e)
        if descending:
            RS.invert_keys(e, key_len)
        if split:
            e[:, 0].bitwise_or_(tag_of(c))
        S.range_dest(e, seps, part_mask)
        return e

    # ---------------------------------------------------------------- 1. count pass
    t0 = time.perf_counter()
    counts = torch.zeros((C, G), dtype=torch.int64, device=dev)
    for c in range(C_local):
        lo, hi = c * chunk_rows, min(n, (c + 1) * chunk_rows)
        if src.dma:
            h2d.wait_stream(comp)          # the previous chunk's extraction has read scratch
        st = src.fill(lo, hi, scratch, h2d)
        if st is not None:
            comp.wait_stream(st)
            stats.bytes_h2d += (hi - lo) * stride
        e = entries(c, scratch[: hi - lo], ent[: hi - lo])
        counts[c] = torch.bincount(e[:, 1], minlength=G)
    allc = shuffle.all_gather_tensor(counts.unsqueeze(0), w).view(W, C, G).cpu()   # [src, chunk, range]
    stats.seconds["count"] = time.perf_counter() - t0

    mine = allc[:, :, me * P:(me + 1) * P]                      # [src, chunk, bucket] rows for me
    rows_b = mine.sum(dim=(0, 1))
    stats.max_bucket = int(rows_b.max()) if P else 0
    if stats.max_bucket > bucket_cap:
        raise RuntimeError(f"external sort: a range bucket holds {stats.max_bucket} rows > {bucket_cap} "
                           f"(key skew with keep_ties, or too small a sample); raise the HBM budget")
    n_out = int(rows_b.sum())
    # hybrid: the largest suffix of buckets that fits next to the working arena stays in HBM
    res_first = P
    if resident:
        room = budget - work - min(256 << 20, budget // 16)
        acc = 0
        for b in range(P - 1, -1, -1):
            nb_ = int(rows_b[b]) * stride
            if acc + nb_ > room:
                break
            acc += nb_
            res_first = b
    res_rows = int(rows_b[res_first:].sum())
    n_host = n_out - res_rows
    stats.resident_rows, stats.resident_buckets = res_rows, P - res_first
    region = torch.empty((res_rows, stride), dtype=torch.uint8, device=dev) if res_rows else None
    # bucket b's first row in its tier: host buckets [0, res_first), then the resident ones
    base = torch.zeros(P, dtype=torch.int64)
    if res_first > 0:
        hb_ = rows_b[:res_first]
        base[:res_first] = torch.cumsum(hb_, 0) - hb_
    if res_first < P:
        rb_ = rows_b[res_first:]
        base[res_first:] = torch.cumsum(rb_, 0) - rb_
    # position of piece (s, c, b) in its tier: bucket start + rows of earlier chunks + earlier sources
    flat = mine.permute(1, 0, 2).reshape(C * W, P)              # (chunk, src) major order
    piece_pos = (torch.cumsum(flat, 0) - flat + base.unsqueeze(0)).view(C, W, P)
    if out is not None and out.n >= n_host and out.stride == stride:
        out = out.view(n_host)
    elif out_factory is not None:
        out = out_factory(n_host)
        stats.tier = "disk" if getattr(out, "path", None) else "dram"
    else:
        out = HostRows(n_host, stride, key_off, key_len)
    try:
        # ------------------------------------------------------------ 2. partition pass
        t0 = time.perf_counter()
        arena.reset()
        rin = [arena.take((chunk_rows, stride)) for _ in range(2)]
        rout = [arena.take((chunk_rows, stride)) for _ in range(2)]
        ent = arena.take((chunk_rows, 2), torch.int64)
        recv = rout
        if W > 1:
            rmax = int(mine.sum(dim=2).sum(dim=0).max())        # rows received in one round
            recv = []
            for _ in range(2):
                try:
                    recv.append(arena.take((max(rmax, 1), stride)))
                except MemoryError:
                    recv.append(torch.empty((max(rmax, 1), stride), dtype=torch.uint8, device=dev))
        ev_in = [torch.cuda.Event() for _ in range(2)]       # rows_in[k] consumed
        ev_ready = [None, None]                              # rows_in[k] filled (copy stream)
        ev_out = [torch.cuda.Event() for _ in range(2)]      # scatter / exchange of round k done
        ev_d2h = [torch.cuda.Event() for _ in range(2)]      # round k's pieces downloaded
        for k in range(2):
            ev_in[k].record(comp)
            ev_d2h[k].record(d2h)

        def prefetch(c):
            if c >= C_local:
                return
            k = c % 2
            lo, hi = c * chunk_rows, min(n, (c + 1) * chunk_rows)
            if src.dma:
                h2d.wait_event(ev_in[k])
                src.fill(lo, hi, rin[k], h2d)
                ev = torch.cuda.Event()
                ev.record(h2d)
                ev_ready[k] = ev
                stats.bytes_h2d += (hi - lo) * stride
            else:
                src.fill(lo, hi, rin[k], None)
                ev_ready[k] = None

        prefetch(0)
        for c in range(C):
            k = c % 2
            prefetch(c + 1)
            cn = min(n, (c + 1) * chunk_rows) - c * chunk_rows if c < C_local else 0
            if ev_ready[k] is not None:
                comp.wait_event(ev_ready[k])
                ev_ready[k] = None
            comp.wait_event(ev_d2h[k])
            if cn > 0:
                e = entries(c, rin[k][:cn], ent[:cn])
                S.bucket_scatter_rows(e, rin[k][:cn], rout[k], sync=False)
            ev_in[k].record(comp)
            if W > 1:
                sc = allc[me, c].view(W, P).sum(1).tolist()
                rc = allc[:, c, me * P:(me + 1) * P].sum(1).tolist()
                shuffle.alltoallv_bytes(rout[k].view(-1), [x * stride for x in sc], recv[k].view(-1),
                                        [x * stride for x in rc], w)
            # pieces of round c: W == 1 -> bucket b of the local chunk; W > 1 -> (src, bucket).
            # Resident buckets' pieces are copied on the compute stream (the copy engines keep to
            # the PCIe pieces), the others go to their host positions on the download stream.
            pieces = []
            a = 0
            for s_ in range(W):
                for b in range(P):
                    cnt = int(mine[s_, c, b])
                    if cnt:
                        p0 = int(piece_pos[c, s_, b])
                        if b >= res_first:
                            region[p0:p0 + cnt].copy_(recv[k][a:a + cnt], non_blocking=True)
                        else:
                            pieces.append((p0, a, cnt))
                    a += cnt
            ev_out[k].record(comp)
            d2h.wait_event(ev_out[k])
            for p0, a, cnt in pieces:
                _copy(out.rows[p0:p0 + cnt], recv[k][a:a + cnt], d2h)
                stats.bytes_d2h += cnt * stride
            ev_d2h[k].record(d2h)
        torch.cuda.synchronize(dev)
        stats.seconds["partition"] = time.perf_counter() - t0

        # ------------------------------------------------------------ 3. sort each bucket
        t0 = time.perf_counter()
        arena.reset()
        cap = max(2, stats.max_bucket)
        bin_ = [arena.take((cap, stride)) for _ in range(2)]
        bout = [arena.take((cap, stride)) for _ in range(2)]
        ea = arena.take((cap, 2), torch.int64)
        eb = arena.take((cap, 2), torch.int64)
        sizes = [int(x) for x in rows_b.tolist()]
        offs = [int(x) for x in base.tolist()]
        nonres = [b for b in range(res_first) if sizes[b]]
        resb = [b for b in range(res_first, P) if sizes[b]]
        # resident buckets sort through a buffer of their own, so the two slots stay with the host
        # buckets: host bucket j+2 uploads into slot j % 2 while bucket j+1 is sorted and bucket j
        # downloads, and both copy directions stream without a gap (with the slots shared, a
        # resident bucket between two host buckets left one slot to the host buckets and the
        # upload engine idle during every sort: ~41 instead of ~48 GB/s per direction)
        rtmp = None
        if resb and nonres:
            try:
                rtmp = arena.take((cap, stride))
            except MemoryError:
                rtmp = None
        # processing order: host buckets (PCIe round trips) interleaved with resident ones (compute
        # only), so the GPU sorts resident buckets while the copy engines move the others; without
        # the extra buffer the resident buckets go last
        order = []
        if rtmp is not None:
            i_r = 0
            for j, b in enumerate(nonres):
                order.append(b)
                want = ((j + 1) * len(resb)) // max(len(nonres), 1)
                while i_r < want:
                    order.append(resb[i_r])
                    i_r += 1
            order += resb[i_r:]
        else:
            order = nonres + resb
        hosts = [b for b in order if b < res_first]          # host buckets, in processing order
        ev_sorted = [torch.cuda.Event() for _ in range(2)]   # slot k's input consumed
        ev_down = [torch.cuda.Event() for _ in range(2)]     # slot k's output downloaded
        for k in range(2):
            ev_sorted[k].record(comp)
            ev_down[k].record(d2h)
        ev_up = {}

        def upload(j):
            if j >= len(hosts) or j in ev_up:
                return
            b, k = hosts[j], j % 2
            h2d.wait_event(ev_sorted[k])       # the slot's previous bucket has been sorted
            _copy(bin_[k][: sizes[b]], out.rows[offs[b]: offs[b] + sizes[b]], h2d)
            ev = torch.cuda.Event()
            ev.record(h2d)
            ev_up[j] = ev
            stats.bytes_h2d += sizes[b] * stride

        upload(0)
        upload(1)
        j = 0
        for b in order:
            mb = sizes[b]
            hb = RS._range_hi_bounds(seps_hi, me * P + b)
            if b >= res_first:
                rows_r = region[offs[b]: offs[b] + mb]
                if rtmp is None:               # after every host bucket: both slots are free
                    comp.wait_event(ev_down[0])
                    comp.wait_event(ev_down[1])
                res = RS.local_sort_rows(rows_r, rtmp if rtmp is not None else bout[0], ea, eb, key_off, key_len,
                                         hi_bounds=hb, descending=descending)
                rows_r.copy_(res[:mb])
                continue
            k = j % 2
            comp.wait_event(ev_down[k])        # slot k's previous output has left for the host
            comp.wait_event(ev_up.pop(j))
            res = RS.local_sort_rows(bin_[k][:mb], bout[k], ea, eb, key_off, key_len, hi_bounds=hb,
                                     descending=descending)
            ev_sorted[k].record(comp)
            d2h.wait_event(ev_sorted[k])
            _copy(out.rows[offs[b]: offs[b] + mb], res[:mb], d2h)
            ev_down[k].record(d2h)
            stats.bytes_d2h += mb * stride
            upload(j + 2)                      # slot k is free once this bucket is sorted
            upload(j + 1)
            j += 1
        torch.cuda.synchronize(dev)
        stats.seconds["sort"] = time.perf_counter() - t0
    finally:
        del arena
    stats.n_out = n_out
    stats.seconds["total"] = time.perf_counter() - t_all
    if region is not None:
        return TieredRows([out.rows[:n_host], region], stride, key_off, key_len, owners=[out])
    return out


def check_terasort_host(out, chunk_rows: int = 1 << 24, descending: bool = False) -> tuple[int, int, bytes, bytes]:
    """valsort over a host (``HostRows``) or tiered (``TieredRows``) TeraSort table: (hash sum mod
    2^64, order violations incl. chunk and segment boundaries, first key, last key); host rows are
    streamed through HBM in chunks, HBM-resident segments checked in place."""
    from . import terasort as TS
    dev = torch.device("cuda", torch.cuda.current_device())
    acc = torch.zeros(2, dtype=torch.int64, device=dev)
    segs = out.segments if isinstance(out, TieredRows) else ([out.rows[: out.n]] if out.n else [])
    buf = None
    prev, bad, first = None, 0, None
    for seg in segs:
        m = seg.shape[0]
        for a in range(0, m, chunk_rows):
            b = min(m, a + chunk_rows)
            if seg.is_cuda:
                rows = seg[a:b]
            else:
                if buf is None:
                    buf = torch.empty((chunk_rows, seg.shape[1]), dtype=torch.uint8, device=dev)
                _copy(buf[: b - a], seg[a:b], None)
                rows = buf[: b - a]
            TS.check(rows, acc, descending=descending)
            k0 = bytes(seg[a, :TS.KEY_BYTES].cpu().numpy())
            if first is None:
                first = k0
            if prev is not None and (prev < k0 if descending else prev > k0):
                bad += 1
            prev = bytes(seg[b - 1, :TS.KEY_BYTES].cpu().numpy())
    torch.cuda.synchronize(dev)
    h, v = acc.tolist()
    return h & _M64, v + bad, first or b"", prev or b""

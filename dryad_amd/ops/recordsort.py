"""Distributed sort of fixed-width record tables resident in HBM (the OrderBy / RangePartition
vertex programs of the GPU executor).

The reference compiles ``OrderBy(keySel)`` into a sampling stage + ``RangePartition`` (CrossProduct
channels) + ``MergeSort``/``Sort`` (LinqToDryad/DryadLinqQueryGen.cs:2362-2474 CreateRangePartition,
:2476 VisitOrderBy; DryadLinqSampler.cs:38-246).  On one MI355X node this becomes, per rank:

  1. extract   — key bytes -> 16-byte (key, row) entries              [HIP: dr_extract_keys]
  2. sample    — deterministic per-rank sample (seeded by rank = vertex id, so idempotent under
                 re-execution), all-gather, sort, pick world-1 evenly spaced separators
  3. range-dest— per entry key range (W * B ranges, B per destination rank) by binary search of
                 the separators, numbered round-major                       [HIP: dr_range_dest_u128]
  4. pack      — one stable LDS-staged bucket scatter of whole rows into a
                 round-major send buffer                                    [HIP: dr_bucket_scatter_rows]
  5. exchange  — count all-to-all + B payload all-to-all-v rounds over xGMI, all queued up front
                                                                            [RCCL]
  6. local sort— per received key range, while later rounds are in flight: extract + hybrid
                 radix sort + row gather                                    [HIP]

With world size 1 steps 2-5 are skipped.  All buffers are preallocated by the caller so a step does
no HBM allocation (everything stays resident; 288 GB per GPU holds in + out + entries).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import torch

from ..parallel.comm import World, get_world
from ..parallel import shuffle
from . import sort as S
from . import terasort as TSG

# pipelined exchange of the multi-rank sort: key sub-ranges per destination rank (0 = from the
# data size; tests set it) and the target bytes per (source, destination) pair and round
PIPE_SUBS = 0
PIPE_ROUND_BYTES = 1 << 30
# fine-bucket exchange over a materialised table: rows a rank receives per round (~1 GiB: the
# overlapped exchange receives each round into one of OVERLAP_SLOTS small slots) and the slots
OVERLAP_ROUND_BYTES = 1 << 30
OVERLAP_SLOTS = 2
_M64 = (1 << 64) - 1


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

    @staticmethod
    def allocate_pitch128(capacity: int, rec: int, device) -> "SortBuffers":
        """The fine-bucket exchange's working set over a table stored at a 128-byte pitch: rows_in
        [cap, 128] (the input, one aligned HBM line per record; after the send-side pack, the
        receive buffer at the record width), rows_out [cap, rec] (send rows, then the output),
        ent_a [cap] int64 (E64 entries).  The entry sort's ping-pong half lives in rows_out,
        free until the pack.  ~1.25e9 TeraSort rows: 298 GB."""
        cap = int(capacity) + 1024
        rows_out = torch.empty((cap, rec), dtype=torch.uint8, device=device)
        rows_in = torch.empty((cap, 128), dtype=torch.uint8, device=device)
        return SortBuffers(rows_in=rows_in, rows_out=rows_out, ent_a=torch.empty(cap, dtype=torch.int64, device=device),
                           ent_b=torch.empty(0, dtype=torch.int64, device=device))

    @property
    def capacity(self) -> int:
        """Rows a rank can receive: the output's rows, and what rows_in holds at the record width."""
        rec = self.rows_out.shape[1]
        return min(self.rows_out.shape[0], self.rows_in.numel() // rec)

    @property
    def pitch(self) -> int:
        return self.rows_in.shape[1]

    def recv_rows(self) -> torch.Tensor:
        """rows_in as the receive buffer: [capacity, record width] over its flat bytes."""
        rec = self.rows_out.shape[1]
        if self.rows_in.shape[1] == rec:
            return self.rows_in
        cap = self.rows_in.numel() // rec
        return self.rows_in.view(-1)[: cap * rec].view(cap, rec)

    def entry_pair(self, n: int, in_out: bool = False) -> tuple[torch.Tensor, torch.Tensor]:
        """(entries, ping-pong scratch) of n E64 entries.  ``in_out``: the producer wrote the
        entries into rows_out's first n * 8 bytes (pitch-128 sets, multi-rank: the sort's odd
        pass count then ends in ent_a, away from the rows the pack writes)."""
        e64 = self.ent_a.view(-1)
        if self.ent_b.numel() >= n:
            return e64[:n], self.ent_b.view(-1)[:n]
        t = self.rows_out.view(-1)[: n * 8].view(torch.int64)
        return (t, e64[:n]) if in_out else (e64[:n], t)


@dataclass
class SortStats:
    n_in: int = 0
    n_out: int = 0
    rounds: int = 1
    send_counts: list = field(default_factory=list)
    recv_counts: list = field(default_factory=list)
    path: str = ""
    round_send_bytes: list = field(default_factory=list)
    round_recv_bytes: list = field(default_factory=list)
    # HIP events on the compute stream: before the first payload collective is queued, after
    # round b's wait (its rows usable), after the receive side's last kernel; the overlapped
    # exchange also records each round's pack ("pack")
    events: dict = field(default_factory=dict)
    overlap: dict = field(default_factory=dict)       # the overlapped exchange's report

    def exchange_report(self) -> dict:
        """Per-round exchange bytes and arrival times (ms after the first payload round was queued:
        when the compute stream could use round b's rows), and the receive tail after the last
        arrival.  Call after the step has synchronised."""
        ev = self.events
        out = dict(path=self.path, rounds=self.rounds, send_GB=round(sum(self.round_send_bytes) / 1e9, 3),
                   recv_GB=round(sum(self.round_recv_bytes) / 1e9, 3),
                   round_send_MB=[round(b / 1e6, 1) for b in self.round_send_bytes],
                   round_recv_MB=[round(b / 1e6, 1) for b in self.round_recv_bytes])
        if "start" in ev and ev.get("arrive"):
            try:
                ev["done"].synchronize()
                arr = [ev["start"].elapsed_time(e) for e in ev["arrive"]]
                out["round_arrival_ms"] = [round(a, 3) for a in arr]
                out["round_wait_ms"] = [round(b - a, 3) for a, b in zip([0.0] + arr[:-1], arr)]
                if "done" in ev:
                    out["receive_tail_ms"] = round(ev["arrive"][-1].elapsed_time(ev["done"]), 3)
                    out["exchange_to_done_ms"] = round(ev["start"].elapsed_time(ev["done"]), 3)
                if ev.get("entry") is not None:
                    out["send_side_before_exchange_ms"] = round(ev["entry"].elapsed_time(ev["start"]), 3)
                if ev.get("pack"):
                    # the overlapped exchange: round 0 queued once its send rows were packed
                    pk = [ev["start"].elapsed_time(e) for e in ev["pack"]]
                    t0 = ev["entry"].elapsed_time(ev["start"]) if ev.get("entry") is not None else 0.0
                    out["first_round_queued_ms"] = round(t0 + pk[0], 3)
                    out["round_packed_ms"] = [round(x, 3) for x in pk]
            except RuntimeError:          # events not recorded (gloo rehearsal on CPU tensors)
                pass
        if self.overlap:
            out["overlap"] = self.overlap
        return out


def invert_keys(e: torch.Tensor, key_len: int) -> torch.Tensor:
    """Invert the key bits (not the row index / tie bits) of E128 entries in place, so that an
    ascending radix sort of them orders the keys descending (OrderByDescending)."""
    _, _, lo_mask = key_bits(key_len)
    e[:, 1].bitwise_not_()
    if lo_mask:
        e[:, 0].bitwise_xor_(torch.tensor(_as_i64(lo_mask), dtype=torch.int64, device=e.device))
    return e


def local_sort_rows(rows: torch.Tensor, out: torch.Tensor, ent_a: torch.Tensor, ent_b: torch.Tensor,
                    key_off: int, key_len: int, descending: bool = False,
                    hi_bounds: tuple[int, int] | None = None, keys_ready: bool = False,
                    keys_fmt: str = "e128", stats: dict | None = None) -> torch.Tensor:
    """Sort fixed-width ``rows`` by their byte-string key into ``out`` (stable).

    Ascending sorts take the compact path (8-byte entries + run fix-up in the row gather,
    ops/sort.sort_rows_compact); descending sorts, and keys so duplicated that a run of equal
    32-bit windows outgrows the gather's LDS window, take the 16-byte-entry hybrid sort.
    ``hi_bounds`` = known (min, max) of the first 8 key bytes as a big-endian integer (e.g. this
    rank's range-partition bounds); lets the sort skip their common prefix without a pass.
    ``keys_ready``: ``ent_a`` already holds the entries of ``rows`` in ``keys_fmt`` ("e64": the
    compact entries for prefix 0, "e128": ``extract_keys(rows, key_off, key_len)``), emitted by
    the producer (the fused TeraSort generator)."""
    n = rows.shape[0]
    if n == 0:
        return out[:0]
    if not descending and S.compact_sort_ok(rows, key_len):
        r = S.sort_rows_compact(rows, out, ent_a.view(-1), ent_b.view(-1), key_off, key_len, hi_bounds=hi_bounds,
                                keys_ready=keys_ready and keys_fmt == "e64", stats=stats)
        if r is not None:
            return r
        keys_ready = False          # the compact attempt reused ent_a
    if keys_fmt != "e128":
        keys_ready = False
    e = ent_a[:n] if keys_ready else S.extract_keys(rows, key_off, key_len, 0, out=ent_a[:n])
    if descending:
        invert_keys(e, key_len)
    b0, b1, _ = key_bits(key_len)
    # 16-byte entries: the hybrid sort (top-window LSD passes + in-LDS run sort)
    srt = S.sort_entries_hybrid(e, b0, b1, tmp=ent_b[:n], hi_bounds=None if descending else hi_bounds)
    return S.gather_rows(rows, entries=srt, out=out[:n])


def sample_count(n: int, sample_target: int) -> tuple[int, int]:
    """(m, stride) of a rank's sample: ~0.001 of its n keys, at least min(n, 16), at most
    sample_target (reference DryadLinqSampler.cs:38-106)."""
    m = max(1, min(n, max(16, min(sample_target, n // 1000 if n >= 16000 else n))))
    return m, max(1, n // m)


def sample_offset(seed: int, rank: int, stride: int) -> int:
    """First sampled position of a rank: deterministic given (seed, rank), so a re-executed
    vertex draws the same sample (the reference seeds its sampler with the vertex id)."""
    return (seed + rank * 7919) % stride if stride > 1 else 0


def separators_from_samples(allsamp: torch.Tensor, parts: int) -> torch.Tensor:
    """Sort every rank's sample on the GPU and pick ``parts`` - 1 evenly spaced separators."""
    total = allsamp.shape[0]
    scratch = torch.empty_like(allsamp)
    srt = S.sort_entries(allsamp.contiguous(), 0, 128, tmp=scratch)
    pos = torch.tensor([(j * total) // parts for j in range(1, parts)], dtype=torch.int64, device=srt.device)
    return srt.index_select(0, pos).contiguous()


def choose_separators(entries: torch.Tensor, n: int, world: World, lo_mask: int, sample_target: int,
                      seed: int, tmp: torch.Tensor, parts: int | None = None) -> torch.Tensor:
    """Sampler (reference DryadLinqSampler.cs:38-246): per-rank stride sample at ~0.001 (at least
    min(n, 16) keys, at most sample_target), all-gathered, sorted on the GPU, ``parts``-1
    (default world-1) separators at evenly spaced ranks.  Deterministic given (rank, n, seed)."""
    parts = parts or world.size
    m, stride = sample_count(n, sample_target)
    off = sample_offset(seed, world.rank, stride)
    samp = entries[off: off + stride * m: stride][:m].clone()
    # keep only key bits in lo
    samp[:, 0] = samp[:, 0] & _as_i64(lo_mask)
    return separators_from_samples(shuffle.all_gather_varlen(samp, world), parts)


def gen_samples(gen: tuple[int, int], n: int, rank: int, lo_or: int, lo_mask: int, sample_target: int,
                seed: int, device) -> torch.Tensor:
    """``choose_separators``' sample of one rank over gen://terasort records gen[0] .. gen[0] + n - 1,
    generated at the sampled positions (the same entries as sampling a generated entry table)."""
    m, stride = sample_count(n, sample_target)
    samp = TSG.sample_keys(gen[0], gen[1], sample_offset(seed, rank, stride), stride, m, lo_or, device)
    samp[:, 0] = samp[:, 0] & _as_i64(lo_mask)
    return samp


def rank_hi_bounds(seps: torch.Tensor, rank: int) -> tuple[int, int]:
    """(min, max) of key ``hi`` words that range partition ``rank`` can receive."""
    return _range_hi_bounds([int(x) & _M64 for x in seps[:, 1].tolist()], rank)


def _as_i64(v: int) -> int:
    v &= (1 << 64) - 1
    return v - (1 << 64) if v >= (1 << 63) else v


def pipeline_subs(max_rank_bytes: int, world_size: int) -> int:
    """Key sub-ranges per destination rank of the pipelined exchange: about PIPE_ROUND_BYTES per
    (source, destination) pair and round, at least 4 (small jobs run the same pipeline), and
    world * subs <= 256 (one radix digit of bucket ids)."""
    cap = max(1, 256 // world_size)
    if PIPE_SUBS:
        return max(1, min(PIPE_SUBS, cap))
    want = -(-max_rank_bytes // max(1, world_size * PIPE_ROUND_BYTES))
    b = 4
    while b < want:
        b <<= 1
    return min(b, cap)


def fine_subs(max_rank_bytes: int, world_size: int) -> int:
    """Rounds (key sub-ranges per destination) of the fine-bucket exchange over a materialised
    table: about OVERLAP_ROUND_BYTES received per rank and round (each round's send rows are packed
    just before it goes out and it is received into a slot of that size), a power of two, at
    least 4, and world * rounds <= 2048 key ranges."""
    cap = max(1, 2048 // world_size)
    if PIPE_SUBS:
        return max(1, min(PIPE_SUBS, cap))
    want = -(-max_rank_bytes // max(1, OVERLAP_ROUND_BYTES))
    b = 4
    while b < want:
        b <<= 1
    return min(b, cap)


def _range_hi_bounds(seps_hi: list, g: int) -> tuple[int, int]:
    """(min, max) of the key ``hi`` words that key range ``g`` (between separators g-1 and g) holds."""
    lo = seps_hi[g - 1] if g > 0 else 0
    hi = seps_hi[g] if g < len(seps_hi) else (1 << 64) - 1
    return lo, hi


def _sort_keys(rows: torch.Tensor, ent: torch.Tensor, tmp: torch.Tensor, key_off: int, key_len: int,
               hi_bounds, descending: bool = False) -> torch.Tensor:
    """Extract + sort the entries of ``rows`` (row indices relative to ``rows``); returns the
    tensor holding the sorted entries (``ent`` or ``tmp``)."""
    e = S.extract_keys(rows, key_off, key_len, 0, out=ent)
    if descending:
        invert_keys(e, key_len)
        hi_bounds = None
    b0, b1, _ = key_bits(key_len)
    return S.sort_entries_hybrid(e, b0, b1, tmp=tmp, hi_bounds=hi_bounds)


def _agree(err: BaseException | None, w: World, what: str, value: int = 0):
    """Gang agreement before a payload collective: every rank's status in one all-gather; if any
    rank failed, every rank raises GangAgreementError alike (the failing one chaining its own
    error), so no rank is left inside a collective its peers never enter.  Returns the ranks'
    values (e.g. their row counts)."""
    st = shuffle.gang_status(err is None, value, w)
    bad = [r for r, (ok, _) in enumerate(st) if not ok]
    if bad:
        from ..errors import GangAgreementError
        msg = f"{what}: rank(s) {bad} failed before the exchange"
        if err is not None:
            raise GangAgreementError(f"{msg} (rank {w.rank}: {type(err).__name__}: {err})", ranks=bad) from err
        raise GangAgreementError(msg, ranks=bad)
    return [v for _, v in st]


def _check_capacity(n_recv: int, cap: int, w: World):
    """Voted capacity check: every rank learns whether any key range overflows its receive
    buffer BEFORE the payload collectives start; all raise the same non-retryable error (the
    split is deterministic: a re-execution would overflow again)."""
    st = shuffle.gang_status(n_recv <= cap, n_recv - cap, w)
    over = [(r, v) for r, (ok, v) in enumerate(st) if not ok]
    if over:
        from ..errors import GangAgreementError
        raise GangAgreementError(
            "range partition skew: " + ", ".join(f"rank {r} receives {v} rows past its capacity" for r, v in over)
            + " (a run of equal keys larger than one rank's buffer, or ShuffleSlack too small)",
            retryable=False, ranks=[r for r, _ in over])


def fine_rows_ok(rec: int, pitch: int, key_off: int, key_len: int, W: int, n: int, one_rank: bool = False) -> bool:
    """The fine-bucket exchange applies: fixed-width records of 12..128 bytes (a multiple of 4)
    keyed by a byte string of at most 10 bytes anywhere in the record (TeraSort rows: 100 bytes,
    key bytes 0..9), stored back to back or at a 128-byte pitch, 2..64 ranks (sources per merged
    bucket; ``one_rank``: a one-rank world that still exchanges through its communicator)."""
    return ((1 < W or (one_rank and W == 1)) and W <= 64 and rec % 4 == 0 and 12 <= rec <= 128
            and 1 <= key_len <= TSG.KEY_BYTES and 0 <= key_off and key_off + key_len <= rec
            and pitch in (rec, 128) and n < (1 << 31))


_WINDOW = _as_i64(0xFFFFFFFF00000000)


def fine_entries(rows: torch.Tensor, key_off: int, key_len: int, e: torch.Tensor, descending: bool = False,
                 hist: bool = True):
    """E64 entries (key window << 32 | row) of ``rows`` for the fine-bucket exchange, with the
    look-back sort's window histograms; ``descending``: the window bits inverted (and the
    histograms mirrored), so the ascending sort, the separators and the fine buckets of the
    inverted key order the rows descending (ts_tile_merge inverts the key alike)."""
    e, h = S.extract_keys64_tile(rows, key_off, key_len, 0, e, hist=hist)
    if descending:
        e.bitwise_xor_(_WINDOW)
        if h is not None:
            h.copy_(h.view(-1, 4, 256).flip(-1).reshape(-1))
    return e, h


def distributed_sort_rows(bufs: SortBuffers, n: int, key_off: int, key_len: int, world: World | None = None,
                          sample_target: int = 1 << 20, seed: int = 314159,
                          stats: SortStats | None = None, keys_ready: bool = False,
                          hi_bounds: tuple[int, int] | None = None, split_ties: bool = True,
                          keys_fmt: str = "e128", gen: tuple[int, int] | None = None,
                          src: torch.Tensor | None = None, descending: bool = False) -> torch.Tensor:
    """Globally sort the first ``n`` rows of ``bufs.rows_in`` (or of ``src``, a table read in
    place and left intact) across all ranks.

    On return rank r holds, in ``bufs.rows_out[:n_r]``, the r-th key range in ascending order.
    ``bufs.rows_in`` is clobbered (it becomes the receive buffer).  ``keys_ready``: the rows'
    sort entries are already there (``keys_fmt`` "e128": ``bufs.ent_a[:n]``; "e64": E64 entries
    with the producer's window histograms in ``ent_a``, "e64@out": in rows_out's first n * 8
    bytes, see SortBuffers.entry_pair); ``hi_bounds``: known hi range of the local keys.
    ``split_ties``: runs of equal keys may be split over ranks (skew); keeps the global order but
    not the co-location of equal keys, so the planner turns it off (keep_ties) when a consumer
    relies on the output being partitioned by the key.  ``descending`` (OrderByDescending): the
    E128 path with the key bits of the entries inverted (rank 0 receives the largest keys; ties
    stay in (rank, row) order), every received round sorted by its inverted keys.

    Three send sides:
      * fine-bucket exchange over the materialised table (TeraSort rows, the default for such
        tables, ``send_fine_rows``): E64 entries sorted on the top ``fb`` key bits, the rows
        packed into the round-major send buffer in fine-bucket order by one gather from the
        table; the receive side orders each fine bucket in LDS (``merge_received_rounds``).
      * ``gen = (first, seed)``: ``rows_in`` was never written; row i is gen://terasort record
        first + i and the send side generates the records into the send rows in bucket order
        (``pack_gen_fine``; the GenFusedShuffle context property: the read fused with the
        exchange, no input table).
      * any other fixed-width table: E128 entries, range destination, stable LDS bucket scatter of
        the rows, and per received round extract + radix sort + gather (``sort_received_rounds``).

    The sampled separators cut the key space into ``W * B`` ranges, B consecutive ones per
    destination rank; the send buffer is round-major (round b = every rank's b-th range), each
    round one RCCL all-to-all-v, all queued up front.  Rank r receives round b as one contiguous
    block holding ALL rows of its key range b and orders it while rounds b+1.. are in flight,
    writing into the send region under it once that has gone out.  Before any payload collective
    the ranks agree (``_agree``, ``_check_capacity``): a rank whose send side failed, or whose
    key ranges overflow its buffers, stops every rank alike instead of leaving its peers in the
    exchange (reference: the sampler + RangePartition + MergeSort stages of
    DryadLinqQueryGen.cs:2362-2474, CrossProduct channels GraphBuilder.cs:481-504)."""
    w = world or get_world()
    W = w.size
    rec = bufs.rows_out.shape[1]
    pitch = bufs.pitch
    rows = bufs.rows_in[:n, :rec] if src is None else src[:n]
    entry = None
    if stats is not None and bufs.rows_out.is_cuda and w.collective:
        entry = torch.cuda.Event(enable_timing=True)          # the send side's start (exchange_report)
        entry.record()
    if src is not None:
        assert src.shape[1] == rec and gen is None and not keys_ready, "src: [n, record width] rows, no producer keys"
        pitch = rec
    if descending:
        hi_bounds = None              # bounds of the ascending keys
    gen_path = gen is not None and fine_rows_ok(rec, pitch, key_off, key_len, W, n, w.force_collectives) \
        and pitch == rec and not descending and (rec, key_off, key_len) == (TSG.RECORD_BYTES, 0, TSG.KEY_BYTES)
    if gen is not None and not gen_path:
        TSG.generate(bufs.rows_in[:n], gen[0], gen[1])       # the records are needed after all
        gen = None
        if keys_fmt == "gen":
            keys_ready = False
    if not w.collective:
        if src is not None:
            bufs.rows_in[:n].copy_(src[:n])
            rows = bufs.rows_in[:n]
        if pitch != rec:
            if descending:
                raise ValueError("distributed_sort_rows: a 128-byte-pitch table sorts ascending only")
            out = S.sort_rows_pitch128(bufs.rows_in[:n], bufs.rows_out, bufs.ent_a, key_off, key_len,
                                       keys_ready=keys_ready and keys_fmt == "e64")
        else:
            out = local_sort_rows(rows, bufs.rows_out, bufs.ent_a, bufs.ent_b, key_off, key_len,
                                  descending=descending, hi_bounds=hi_bounds, keys_ready=keys_ready,
                                  keys_fmt=keys_fmt)
        if stats is not None:
            stats.n_in = stats.n_out = n
            stats.path = "local"
        return out
    fine_rows = gen is None and fine_rows_ok(rec, pitch, key_off, key_len, W, n, w.force_collectives)
    if descending and keys_fmt != "e128":
        keys_ready = False              # a producer's entries hold the ascending key
    if pitch != bufs.pitch and not fine_rows:
        raise ValueError("distributed_sort_rows: a src table needs a buffer set at its record width")
    if pitch != rec and not fine_rows:
        raise ValueError(f"distributed_sort_rows: a {pitch}-byte-pitch table needs the fine-bucket exchange")
    _, _, lo_mask = key_bits(key_len)
    split = split_ties and key_len <= 10 and W < (1 << 16)
    # skew: equal keys must not all land on one rank.  Bits 47..32 of lo are free for keys of
    # <= 10 bytes; with the rank there (and the row index below it) every entry is unique, so the
    # sampled separators split runs of equal keys across ranks while the global order (key, rank,
    # row) stays a valid OrderBy order.  (The fine-bucket paths cut separators to bucket edges:
    # equal keys stay on one rank there.)
    part_mask = _M64 if split else lo_mask
    lo_or = (w.rank << 32) if split else 0
    err = None
    samp = None
    try:
        if gen_path:
            samp = gen_samples(gen, n, w.rank, lo_or, part_mask, sample_target, seed, w.device)
        elif fine_rows:
            in_out = keys_ready and keys_fmt == "e64@out"
            e, tmp = bufs.entry_pair(n, in_out=in_out)
            hist = S.take_gen_hist(e) if keys_ready and keys_fmt in ("e64", "e64@out") else None
            if hist is None and not (keys_ready and keys_fmt in ("e64", "e64@out")):
                e, hist = fine_entries(rows, key_off, key_len, e, descending)
            samp = e64_samples(e, n, w.rank, sample_target, seed)
        else:
            if keys_fmt != "e128":
                keys_ready = False
            ent = bufs.ent_a[:n] if keys_ready else S.extract_keys(rows, key_off, key_len, 0, out=bufs.ent_a[:n])
            if descending:
                invert_keys(ent, key_len)
            if split:
                ent[:, 0].bitwise_or_(lo_or)
    except Exception as ex:  # noqa: BLE001
        err = ex
    nmax = max(_agree(err, w, "distributed OrderBy (entries)", n))
    B = fine_subs(nmax * rec, W) if fine_rows else pipeline_subs(nmax * rec, W)
    pack = None
    fine = None
    plan = None
    try:
        if gen_path or fine_rows:
            seps = separators_from_samples(shuffle.all_gather_varlen(samp, w), W * B)
            fb = fine_bits(nmax * W)
            seps_hi = [int(x) & _M64 for x in seps[:, 1].tolist()]
            if fine_rows and _fine_collapsed(seps_hi, fb) and bufs.ent_b.numel() >= 2 * n and pitch == rec:
                # two separators inside one fine bucket: heavy duplication, or keys whose leading
                # bits hardly vary.  The fine cut would give the whole bucket to one rank (and
                # overflow the LDS merge); the E128 path cuts at full key resolution and, with
                # split ties, splits runs of equal keys (key, rank, row).  The separators are
                # global, so every rank switches alike.
                fine_rows = False
                B = pipeline_subs(nmax * rec, W)        # (the E128 path: world * rounds <= 256)
                ent = S.extract_keys(rows, key_off, key_len, 0, out=bufs.ent_a[:n])
                if descending:
                    invert_keys(ent, key_len)
                ent[:, 0].bitwise_or_(lo_or)
                seps = choose_separators(ent, n, w, part_mask, sample_target, seed, bufs.ent_b, parts=W * B)
                seps_hi = [int(x) & _M64 for x in seps[:, 1].tolist()]
            elif gen_path:
                st, pack, counts, L = pack_gen_fine(bufs, gen, n, seps_hi, B, W, fb)
            if fine_rows:
                # the rows are packed round by round in the exchange below, each just before it goes out
                plan = FineSend(bufs, rows, e, tmp, hist, n, seps_hi, B, W, fb,
                                rebuild=lambda: fine_entries(rows, key_off, key_len, e, descending, hist=False)[0])
                st, counts, L = plan.st, plan.counts, plan.L
        else:
            seps = choose_separators(ent, n, w, part_mask, sample_target, seed, bufs.ent_b, parts=W * B)
            seps_hi = [int(x) & _M64 for x in seps[:, 1].tolist()]
    except Exception as ex:  # noqa: BLE001
        err = ex
    else:
        err = None
    if err is None and not (gen_path or fine_rows):
        # (choose_separators holds a collective: the agreement after it covers range_dest + scatter)
        try:
            S.range_dest(ent, seps, part_mask, subs=B, ranks=W)                  # ent.hi := b * W + rank
            st = S.bucket_scatter_rows(ent, rows, bufs.rows_out)                # send buffer, round-major
        except Exception as ex:  # noqa: BLE001
            err = ex
    _agree(err, w, "distributed OrderBy (send side)")
    if gen_path or fine_rows:
        fine = exchange_fine_counts(counts, L, B, W, w)
    send = [[st[b * W + r + 1] - st[b * W + r] for r in range(W)] for b in range(B)]
    sc = torch.tensor([[send[b][r] for b in range(B)] for r in range(W)], dtype=torch.int64)
    rc = shuffle.exchange_counts(sc.flatten(), w).view(W, B).tolist()    # rc[src][b]
    off = [0]
    for b in range(B):
        off.append(off[-1] + sum(rc[s][b] for s in range(W)))
    n_recv = off[-1]
    # a rank whose key ranges outgrow its buffers (skew past ShuffleSlack, e.g. runs of equal keys
    # kept together) receives into buffers of its own when HBM allows; the vote below stops every
    # rank cleanly when it does not
    rb, n_sent = bufs, n
    if n_recv > bufs.capacity:
        try:
            rb = SortBuffers.allocate(n_recv, rec, bufs.rows_out.device)
            n_sent = 0                      # the output no longer overlays the send rows
        except Exception:  # noqa: BLE001 (out of HBM: the capacity vote reports it)
            rb = bufs
    _check_capacity(n_recv, rb.capacity, w)
    ev = {}
    if stats is not None and bufs.rows_out.is_cuda:
        ev = dict(start=torch.cuda.Event(enable_timing=True), done=torch.cuda.Event(enable_timing=True),
                  arrive=[torch.cuda.Event(enable_timing=True) for _ in range(B)], entry=entry)
        ev["start"].record()
    if plan is not None:
        ov = _overlapped_fine_exchange(plan, rb, bufs, off, send, rc, fine, fb, B, W, w, n_sent, ev, key_off, key_len,
                                       descending)
        if ov is None:                 # no room for the receive slots: pack everything, then exchange
            for b in range(B):
                plan.pack(b)
        else:
            out, ov_stats = ov
    if plan is None or ov is None:
        out = _bulk_exchange(bufs, rb, st, send, off, rc, B, W, w, pack, fine, L if fine is not None else None,
                             fb if fine is not None else 0, n_sent, ev, seps_hi, key_off, key_len, descending)
    if ev:
        ev["done"].record()
    if plan is not None and int(plan.bad.item()):
        raise RuntimeError("fine-bucket send side: an entry named a row past the table (corrupt entries)")
    if stats is not None:
        stats.n_in, stats.n_out, stats.rounds = n, n_recv, B
        stats.send_counts = [sum(send[b][r] for b in range(B)) for r in range(W)]
        stats.recv_counts = [sum(rc[s]) for s in range(W)]
        stats.path = ("fine-bucket exchange, records generated into the send rows" if gen_path else
                      f"fine-bucket exchange over the table (pitch {pitch}), "
                      + ("rounds packed as they go out, received into slots" if plan is not None and ov is not None
                         else "table packed before the first round") if fine_rows else
                      "E128 range partition + per-round radix sort")
        stats.round_send_bytes = [(st[(b + 1) * W] - st[b * W] - send[b][w.rank]) * rec for b in range(B)]
        stats.round_recv_bytes = [(off[b + 1] - off[b] - rc[w.rank][b]) * rec for b in range(B)]
        stats.events = ev
        if plan is not None and ov is not None:
            stats.overlap = ov_stats
    return out[:n_recv]


def _bulk_exchange(bufs, rb, st, send, off, rc, B, W, w, pack, fine, L, fb, n_sent, ev, seps_hi, key_off, key_len,
                   descending):
    """Every payload round queued up front, the send rows complete before the first (the receive
    buffer is the input table's memory, rows_in); each round ordered as it arrives."""
    rec = bufs.rows_out.shape[1]
    recv_rows = rb.recv_rows()
    send_flat, recv_flat = bufs.rows_out.view(-1), recv_rows.view(-1)
    handles = []
    for b in range(B):
        if pack is not None:
            pack(b)                    # round b's rows packed (compute stream) before it is queued
        handles.append(shuffle.alltoallv_bytes_async(
            send_flat[st[b * W] * rec: st[(b + 1) * W] * rec], [c * rec for c in send[b]],
            recv_flat[off[b] * rec: off[b + 1] * rec], [rc[s][b] * rec for s in range(W)], w))

    def wait(b):
        shuffle.wait(handles[b])
        if ev:
            ev["arrive"][b].record()
    sent_after = [st[(b + 1) * W] for b in range(B)]
    if fine is not None:
        return merge_received_rounds(rb, off, fine, L, fb, B, w.rank, sent_after, n_sent, wait=wait, key_off=key_off,
                                     key_len=key_len, descending=descending)
    return sort_received_rounds(rb, off, sent_after, n_sent, seps_hi, B, w.rank, key_off, key_len, wait=wait,
                                descending=descending)


def overlap_schedule(st: list, off: list, B: int, W: int, n_sent: int, slots: int):
    """When each received round of the overlapped exchange may be merged: k[j] = the last payload
    round that must have completed before round j's rows are written to out[off[j]:off[j+1]]
    (its own arrival, and the send rows under that output having gone out; rows past ``n_sent``
    never held send data).  None when some round would hold its slot past ``slots`` rounds (the
    receive slots would be overwritten before the merge read them)."""
    k = []
    for j in range(B):
        need = min(off[j + 1], n_sent)
        kk = j
        while kk < B - 1 and st[(kk + 1) * W] < need:
            kk += 1
        k.append(kk)
        if kk > j + slots - 1:
            return None
    return k


def overlap_model(t_ready: float, pack_ms: list, merge_ms: list, wire_ms: list, sched: list | None, slots: int,
                  bulk: bool = False) -> dict:
    """Timeline of the fine-bucket exchange from per-round kernel and link times (ms): one compute
    stream (packs, merges) and one communicator stream (rounds in order; a round starts when
    everything queued before it on the compute stream is done, as RCCL's stream waits on the
    caller's).  ``bulk``: every round packed before the first goes out (the table is the
    receive buffer).  Used to MODEL a node's step from one-GPU measurements (bench.py
    --loopback-ranks --model-link-GBps)."""
    B = len(pack_ms)
    sched = sched if sched is not None else list(range(B))
    comp, comm = t_ready, 0.0
    end = [0.0] * B
    first = None
    idle, last_end = 0.0, None

    def coll(i, ready):
        nonlocal comm, idle, last_end
        start = max(ready, comm)
        if last_end is not None:
            idle += max(0.0, start - last_end)
        end[i] = start + wire_ms[i]
        comm = last_end = end[i]

    def merge(j):
        nonlocal comp
        comp = max(comp, end[sched[j]]) + merge_ms[j]
    if bulk:
        comp += sum(pack_ms)
        first = comp
        for i in range(B):
            coll(i, comp)
        for j in range(B):
            merge(j)
    else:
        pending = list(range(B))
        for i in range(B):
            comp += pack_ms[i]
            if first is None:
                first = comp
            coll(i, comp)
            while pending and (sched[pending[0]] <= i - 1 or pending[0] <= i + 1 - slots):
                merge(pending.pop(0))
        while pending:
            merge(pending.pop(0))
    return dict(step_ms=comp, first_queued_ms=first, wire_idle_ms=idle, wire_end_ms=comm)


def _overlapped_fine_exchange(plan, rb, bufs, off, send, rc, fine, fb, B, W, w, n_sent, ev, key_off, key_len,
                              descending=False):
    """The fine-bucket exchange with the send side overlapped: round i's send rows are packed
    (plan.pack(i)) just before its all-to-all-v is queued, so the first round is on the wire after
    1/B of the pack instead of all of it.  The input table must stay readable until the last pack,
    so nothing is received into it: round i lands in receive slot i % OVERLAP_SLOTS (each the size
    of the largest round; the table's free tail holds what fits, the rest is allocated) and is merged from there into its final place out[off[i]:off[i+1]] (the
    output overlays the send rows: the merge waits until the rows under it have gone out,
    ``overlap_schedule``).  Queue order per round i: pack(i), all-to-all-v(i) [the communicator's
    stream waits for everything queued before it on the compute stream, so a slot is reused only
    after the merge that read it], then the merges that are safe.  Returns (output rows, report),
    or None when the slots do not fit in HBM (the caller packs everything and uses the bulk path)."""
    rec = bufs.rows_out.shape[1]
    NS = OVERLAP_SLOTS
    out_buf = rb.rows_out
    sched = overlap_schedule(plan.st, off, B, W, n_sent if rb is bufs else 0, NS)
    if sched is None:
        return None
    slot_rows = max([off[b + 1] - off[b] for b in range(B)] + [1])
    # receive slots: the buffer set's free input memory holds as many as fit (rows_in past the
    # table: the capacity slack, ~1.6 GB at 125 GB per rank; all of rows_in when the table is read
    # in place from elsewhere), the rest are allocated
    flat_in = bufs.rows_in.view(-1)
    tail = flat_in[plan.rows.shape[0] * bufs.rows_in.shape[1]:] if plan.rows.data_ptr() == flat_in.data_ptr() \
        else flat_in
    in_tail = min(NS, tail.numel() // max(1, slot_rows * rec))
    try:
        extra = torch.empty(((NS - in_tail) * slot_rows, rec), dtype=torch.uint8, device=out_buf.device) \
            if in_tail < NS else None
    except (torch.OutOfMemoryError, RuntimeError):
        return None
    slot_t = [tail[i * slot_rows * rec: (i + 1) * slot_rows * rec].view(slot_rows, rec) for i in range(in_tail)]
    slot_t += [extra[i * slot_rows: (i + 1) * slot_rows] for i in range(NS - in_tail)]
    merger = FineMerge(fine, plan.L, fb, B, w.rank, out_buf, key_off, key_len, descending)
    cuda = out_buf.is_cuda
    flags_host = torch.zeros(B, dtype=torch.int32, pin_memory=cuda)
    merged_ev = [None] * B
    tev = dict(pack=[], queued=None) if ev else None
    handles = [None] * B
    pending = list(range(B))           # rounds not merged yet, in order
    send_flat = bufs.rows_out.view(-1)
    fixups = []

    def merge(j: int):
        for h in range(j, sched[j] + 1):
            shuffle.wait(handles[h])
        if ev:
            ev["arrive"][j].record()
        merger.merge(j, slot_t[j % NS], 0, off[j], off[j + 1])
        if cuda:
            flags_host[j: j + 1].copy_(merger.flags[j: j + 1], non_blocking=True)
            merged_ev[j] = torch.cuda.Event()
            merged_ev[j].record()
        else:
            flags_host[j] = merger.flags[j]

    def check(j: int):
        """Before slot j % NS is received into again: a round whose bucket outgrew LDS is ordered
        from the slot now (rare: heavy key skew), while its rows are still there."""
        if merged_ev[j] is not None:
            merged_ev[j].synchronize()
        if int(flags_host[j]):
            a, z = off[j], off[j + 1]
            ea = torch.empty((z - a, 2), dtype=torch.int64, device=out_buf.device)
            eb = torch.empty_like(ea)
            local_sort_rows(slot_t[j % NS][: z - a], out_buf[a:z], ea, eb, key_off, key_len, descending=descending,
                            hi_bounds=None if descending else fine_hi_bounds(plan.L, fb, w.rank * B + j))
            fixups.append(j)

    for i in range(B):
        plan.pack(i)
        if ev:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            tev["pack"].append(e)
        if i >= NS:
            check(i - NS)
        a, z = plan.st[i * W], plan.st[(i + 1) * W]
        handles[i] = shuffle.alltoallv_bytes_async(
            send_flat[a * rec: z * rec], [c * rec for c in send[i]],
            slot_t[i % NS].view(-1)[: (off[i + 1] - off[i]) * rec], [rc[s][i] * rec for s in range(W)], w)
        # merges whose inputs and output rows are ready without waiting for round i, and the one
        # whose slot round i + 1 needs (which may wait for round i)
        while pending and (sched[pending[0]] <= i - 1 or pending[0] <= i + 1 - NS):
            merge(pending.pop(0))
    while pending:
        merge(pending.pop(0))
    for j in range(max(0, B - NS), B):
        check(j)
    report = dict(mode="rounds packed as they go out", slots=NS, slot_GB=round(slot_rows * rec / 1e9, 3),
                  slots_in_table_tail=in_tail, merge_after=[k - j for j, k in enumerate(sched)], skew_fixups=fixups)
    if ev:
        ev["pack"] = tev["pack"]
    del slot_t, extra
    return out_buf[: off[-1]], report


def _fine_collapsed(seps_hi: list, fb: int) -> bool:
    """Two separators fall into one fine bucket (some key range would be empty and one bucket
    would carry a whole range's share of rows): heavily duplicated keys."""
    L = fine_bounds(seps_hi, fb)
    return any(L[g] == L[g + 1] for g in range(1, len(L) - 2))


def e64_samples(e: torch.Tensor, n: int, rank: int, sample_target: int, seed: int) -> torch.Tensor:
    """``choose_separators``' sample of one rank taken from its E64 entries (key bytes 0..3 in the
    high word): [m, 2] int64 sample entries whose hi word holds those key bits.  The fine-bucket
    exchange cuts separators to the top fb <= 24 key bits, which the window holds."""
    m, stride = sample_count(n, sample_target)
    off = sample_offset(seed, rank, stride)
    w = e[off: off + stride * m: stride][:m]
    samp = torch.zeros((w.shape[0], 2), dtype=torch.int64, device=e.device)
    samp[:, 1] = w & _as_i64(0xFFFFFFFF00000000)
    return samp


class FineSend:
    """Send side of the fine-bucket exchange over a materialised table (``rows``: [n, 100] at a
    100- or 128-byte pitch): one look-back sort of the rows' E64 entries ``e`` (window = key bytes
    0..3, with the producer's / extraction's histograms ``hist``) on the top 8 * ceil(fb / 8) key
    bits, the fine-bucket starts of the sorted order, the send-row starts ``st[b * W + r]`` of the
    round-major send buffer ``bufs.rows_out`` (round b = key range r * B + b for every destination
    r, each piece in fine-bucket order), the per-bucket row counts ``counts`` (device int32 [2^fb])
    and the fine bounds ``L``.  ``pack(b)`` gathers round b's rows from the table into the send
    buffer (ts_pack_rows: 16-byte loads, one HBM line per row at pitch 128), so the exchange can
    send round b while later rounds are still being packed.  A failed look-back sort is redone
    with count + scatter passes over ``rebuild()``'s entries before anything is packed."""

    def __init__(self, bufs: SortBuffers, rows: torch.Tensor, e: torch.Tensor, tmp: torch.Tensor, hist, n: int,
                 seps_hi: list, B: int, W: int, fb: int, rebuild=None, group: int = 1):
        err = S.lookback_error()
        win = 8 * ((fb + 7) // 8)
        srt = S.sort_entries64(e, tmp, win, gen_hist=hist, err=err)
        starts = TSG.fine_starts(srt, fb)
        L = fine_bounds(seps_hi, fb)
        Lt = torch.tensor(L, dtype=torch.int64, device=e.device)
        host = torch.cat([starts.index_select(0, Lt).to(torch.int64), err.to(torch.int64)]).tolist()
        Sg = host[:-1]
        if host[-1]:              # the look-back sort gave up: entries again, count + scatter passes
            e2 = rebuild() if rebuild is not None else e
            srt = S.sort_entries64(e2, tmp if e2.data_ptr() == e.data_ptr() else e, win, lookback=False)
            starts = TSG.fine_starts(srt, fb)
            Sg = starts.index_select(0, Lt).tolist()
            err = None
        self.counts = starts[1:] - starts[:-1]
        st, acc = [], 0
        for b in range(B):
            for r in range(W):
                st.append(acc)
                acc += Sg[r * B + b + 1] - Sg[r * B + b]
        st.append(acc)
        if srt.data_ptr() == bufs.rows_out.data_ptr():
            # (an even pass count left the entries in rows_out, which the pack writes: move them)
            e64 = bufs.ent_a.view(-1)[:n] if bufs.ent_a.data_ptr() != srt.data_ptr() else None
            if e64 is None or e64.numel() < n:
                raise RuntimeError("send_fine_rows: no room for the sorted entries outside the send buffer")
            e64.copy_(srt)
            srt = e64
        # per round: W segments {send row relative to the round's start, first sorted entry}
        self.segs = torch.tensor([[st[b * W + r] - st[b * W], Sg[r * B + b]] for b in range(B) for r in range(W)],
                                 dtype=torch.int64).to(e.device)
        self.bufs, self.rows, self.srt, self.err = bufs, rows, srt, err
        self.st, self.L, self.Sg, self.B, self.W = st, L, Sg, B, W
        self.bad = torch.zeros(1, dtype=torch.int32, device=e.device)
        # rounds per pack launch (``group``): round b is packed with the first round of its group
        self.group = max(1, min(int(group), 256 // max(W, 1)))
        if self.group > 1:
            g = self.group
            self.gsegs = torch.tensor([[st[b * W + r] - st[(b // g) * g * W], Sg[r * B + b]]
                                       for b in range(B) for r in range(W)], dtype=torch.int64).to(e.device)

    def pack(self, b: int) -> None:
        """Round b's send rows: out[st[b * W]: st[(b + 1) * W]] gathered from the table (with
        ``group`` > 1, rounds b .. b + group - 1 in one launch when b starts a group)."""
        W, g = self.W, self.group
        if b % g:
            return
        e = min(self.B, b + g)
        a, z = self.st[b * W], self.st[e * W]
        if z > a:
            segs = self.segs[b * W: e * W] if g == 1 else self.gsegs[b * W: e * W]
            TSG.pack_rows(self.bufs.rows_out[a:z], self.rows, self.srt, z - a, seg=segs, err=self.err, bad=self.bad)


def send_fine_rows(bufs: SortBuffers, rows: torch.Tensor, e: torch.Tensor, tmp: torch.Tensor, hist, n: int,
                   seps_hi: list, B: int, W: int, fb: int, rebuild=None):
    """The whole send side at once (FineSend, then every round packed): (send-row starts
    st[b * W + r], per-bucket row counts, fine bounds L, the pack's bad-entry flag)."""
    plan = FineSend(bufs, rows, e, tmp, hist, n, seps_hi, B, W, fb, rebuild=rebuild)
    for b in range(B):
        plan.pack(b)
    return plan.st, plan.counts, plan.L, plan.bad


# Fine buckets of the gen:// exchange: the top ``fb`` key bits, about FINE_ROWS rows of the whole
# job each (at most tile_cap() = 1024 are ordered by one workgroup); 16 <= fb <= 24, so the send
# side's sort needs at most three 8-bit look-back passes and a bucket's remaining key bits fit
# one 64-bit word.
FINE_MIN_BITS, FINE_MAX_BITS, FINE_ROWS = 16, 24, 600


def fine_bits(total_rows: int) -> int:
    fb = FINE_MIN_BITS
    while fb < FINE_MAX_BITS and total_rows > FINE_ROWS * (1 << fb):
        fb += 1
    return fb


def fine_bounds(seps_hi: list, fb: int) -> list:
    """L[g] = first fine bucket of key range g (g = 0 .. len(seps_hi) + 1): each separator cut
    down to a bucket edge, so a key range is a union of whole fine buckets."""
    return [0] + [int(x) >> (64 - fb) for x in seps_hi] + [1 << fb]


def fine_hi_bounds(L: list, fb: int, g: int) -> tuple[int, int]:
    """(min, max) of the key ``hi`` words key range ``g`` of fine bounds ``L`` holds."""
    return L[g] << (64 - fb), min((L[g + 1] << (64 - fb)) - 1, _M64)


def pack_gen_fine(bufs: SortBuffers, gen: tuple[int, int], n: int, seps_hi: list, B: int, W: int, fb: int):
    """Send side over gen://terasort records gen[0] .. gen[0] + n - 1 for the fine-bucket exchange:
    E64 entries from the generator (key bytes 0..3 as the window, with the look-back sort's digit
    histograms), one look-back sort of them on the top 8 * ceil(fb / 8) key bits (stable), the
    fine-bucket starts of the sorted order.
    Key range g = fine buckets [L[g], L[g + 1]) is then the contiguous run of sorted entries
    [S[L[g]], S[L[g + 1]]), and the send buffer (``bufs.rows_out``) is packed round-major (round b
    = range r * B + b for every destination r), each range's records generated in key order
    (bucket order; unsorted within a bucket).  Returns (send-row starts st[b * W + r] as a host
    list, pack(b), the per-bucket row counts (device int32 [2^fb]), L).  The sorted entries live in
    ``bufs.ent_a`` / ``ent_b`` until the last pack."""
    e, tmp = bufs.ent_a.view(-1)[:n], bufs.ent_b.view(-1)[:n]
    hist = TSG.gen_entries64(e, gen[0], gen[1])
    err = S.lookback_error()
    win = 8 * ((fb + 7) // 8)
    srt = S.sort_entries64(e, tmp, win, gen_hist=hist, err=err)
    starts = TSG.fine_starts(srt, fb)
    L = fine_bounds(seps_hi, fb)
    Lt = torch.tensor(L, dtype=torch.int64, device=e.device)
    host = torch.cat([starts.index_select(0, Lt).to(torch.int64), err.to(torch.int64)]).tolist()
    Sg = host[:-1]
    if host[-1]:                 # the look-back sort gave up: entries again, count + scatter passes
        TSG.gen_entries64(e, gen[0], gen[1], hist=False)
        srt = S.sort_entries64(e, tmp, win, lookback=False)
        starts = TSG.fine_starts(srt, fb)
        Sg = starts.index_select(0, Lt).tolist()
    counts = starts[1:] - starts[:-1]
    size = [[Sg[r * B + b + 1] - Sg[r * B + b] for r in range(W)] for b in range(B)]
    st, acc = [], 0
    for b in range(B):
        for r in range(W):
            st.append(acc)
            acc += size[b][r]
    st.append(acc)

    # generator launches over groups of rounds 1, 1, 2, 4, ... (at most 64 // W rounds, the segment
    # limit): round 0 goes out after 1/B of the pack, and the pack is a handful of launches (16
    # per-round launches cost 27.1 ms against 21.3 ms for one, profiles/r4/send_ab2.log).
    # Segment = {send row - group start, first sorted entry} per (round, destination).
    groups, b0, size_g = [], 0, 1
    while b0 < B:
        g1 = min(B, b0 + size_g, b0 + max(1, 64 // W))
        groups.append((b0, g1))
        if b0 > 0:
            size_g *= 2
        b0 = g1
    segs = torch.tensor([[st[b * W + r] - st[g0 * W], Sg[r * B + b]] for g0, g1 in groups for b in range(g0, g1)
                         for r in range(W)], dtype=torch.int64).to(e.device)
    first_seg = {}
    k = 0
    for g0, g1 in groups:
        first_seg[g0] = (g1, k)
        k += (g1 - g0) * W

    def pack(b: int):
        if b not in first_seg:
            return                   # packed with the first round of its group
        g1, k0 = first_seg[b]
        a, z = st[b * W], st[g1 * W]
        if z > a:
            TSG.gen_gather64(bufs.rows_out[a:z], srt, gen[0], gen[1], seg=segs[k0: k0 + (g1 - b) * W], n=z - a)
    return st, pack, counts, L


def exchange_fine_counts(counts: torch.Tensor, L: list, B: int, W: int, world: World) -> torch.Tensor:
    """Every source's per-bucket row counts of this rank's key ranges: int32 [W, K] (K = buckets
    of ranges rank * B .. rank * B + B - 1, which are contiguous in every source's counts)."""
    me = world.rank
    K = L[(me + 1) * B] - L[me * B]
    recv = torch.empty(W * K, dtype=torch.int32, device=counts.device)
    shuffle.alltoallv_bytes(counts.contiguous().view(torch.uint8), [(L[(r + 1) * B] - L[r * B]) * 4 for r in range(W)],
                            recv.view(torch.uint8), [K * 4] * W, world)
    return recv.view(W, K)


class FineMerge:
    """Receive side of the fine-bucket exchange, one round at a time.  ``fine[s, k]`` = rows of
    bucket L[rank * B] + k from source s; a received round b (key range g = rank * B + b) is W
    source pieces in source order, each in bucket order.  ``merge(b, recv, base, a, z)``: the
    round's rows are ``recv[base: base + z - a]``; the slices of every bucket are located on the
    device (prefix sums of ``fine``) and ts_tile_merge orders each bucket in LDS into
    ``out[a:z]`` by the key spec (``key_off``, ``key_len``, ``descending``).  A bucket too large
    for LDS (heavy key skew) sets ``flags[b]``."""

    def __init__(self, fine: torch.Tensor, L: list, fb: int, B: int, rank: int, out: torch.Tensor,
                 key_off: int = 0, key_len: int = 10, descending: bool = False):
        self.W, self.K = fine.shape
        W, K = self.W, self.K
        self.key = dict(key_off=key_off, key_len=key_len, descending=descending)
        # every key bit is a bucket bit: a bucket holds one key, its merge is a copy in source
        # order at any size (long runs of equal keys would overflow the LDS merge)
        self.whole = 8 * key_len <= fb
        self.L, self.fb, self.B, self.rank, self.out = L, fb, B, rank, out
        dev = out.device
        self.flags = torch.zeros(B, dtype=torch.int32, device=dev)
        self.base = L[rank * B]
        # Every round's merge arguments computed once, up front, in a handful of device passes
        # (per round only slices remain: one kernel launch per round).  Round b holds buckets
        # [k0_b, k1_b); a bucket's slice from source s starts at
        #   pre[s, k] = (rows of s before k in the round) + (rows of sources < s in the round)
        # relative to the round's first received row, and its output at
        #   outoff[k] = (rows of all sources before k in the round) relative to the round's output.
        # Both are laid out round-major ([W, k1_b - k0_b] blocks back to back), so a round's
        # arguments are contiguous slices.
        fine = fine.contiguous()
        kb = torch.tensor([L[rank * B + b] - self.base for b in range(B + 1)], dtype=torch.int64, device=dev)
        self.kb = [L[rank * B + b] - self.base for b in range(B + 1)]
        if K == 0:                       # this rank's key ranges hold no bucket (e.g. all keys equal)
            self.pre = torch.zeros(0, dtype=torch.int64, device=dev)
            self.cnt = torch.zeros(0, dtype=fine.dtype, device=dev)
            self.outoff = torch.zeros(0, dtype=torch.int64, device=dev)
            return
        assert self.kb[0] == 0 and self.kb[-1] == K, (self.kb[0], self.kb[-1], K)
        ex = torch.cumsum(fine.view(-1), 0, dtype=torch.int64).view(W, K) - fine
        ex = ex - ex[:, :1]                                   # rows of source s before bucket k
        ext = torch.cat([ex, fine.sum(1, keepdim=True, dtype=torch.int64)], 1)     # [W, K + 1]
        rid = torch.bucketize(torch.arange(K, dtype=torch.int64, device=dev), kb[1:], right=True)
        rows_per_src = ext[:, kb[1:]] - ext[:, kb[:-1]]                              # [W, B]
        src_base = torch.cumsum(rows_per_src, 0) - rows_per_src                     # [W, B]
        pre_rel = ex - ext[:, kb[:-1]][:, rid] + src_base[:, rid]                   # [W, K]
        col = fine.sum(0, dtype=torch.int64)
        cex = torch.cumsum(col, 0) - col
        self.outoff = (cex - cex[kb[:-1]][rid]).contiguous()                          # [K]
        # round-major blocks: element (s, k) of round b at W * k0_b + s * (k1_b - k0_b) + (k - k0_b)
        k0 = kb[:-1][rid]
        width = (kb[1:] - kb[:-1])[rid]
        kk = torch.arange(K, dtype=torch.int64, device=dev)
        pos = (W * k0 + (kk - k0)).unsqueeze(0) + torch.arange(W, dtype=torch.int64, device=dev).unsqueeze(1) * width
        self.pre = torch.empty(W * K, dtype=torch.int64, device=dev).scatter_(0, pos.view(-1), pre_rel.view(-1))
        self.cnt = torch.empty(W * K, dtype=fine.dtype, device=dev).scatter_(0, pos.view(-1), fine.view(-1))

    def merge(self, b: int, recv: torch.Tensor, base: int, a: int, z: int) -> None:
        """Round b: its rows ``recv[base: base + z - a]`` -> ``out[a:z]`` (one kernel launch)."""
        if z <= a:
            return
        k0, k1 = self.kb[b], self.kb[b + 1]
        W = self.W
        pre = self.pre[W * k0: W * k1].view(W, k1 - k0)
        cnt = self.cnt[W * k0: W * k1].view(W, k1 - k0)
        if self.whole:
            TSG.bucket_copy(recv[base:], self.out[a:], pre, cnt, self.outoff[k0:k1])
        else:
            TSG.tile_merge(recv[base:], self.out[a:], pre, cnt, self.outoff[k0:k1], self.fb, self.flags[b:b + 1],
                           **self.key)


def merge_received_rounds(bufs: SortBuffers, off: list, fine: torch.Tensor, L: list, fb: int, B: int, rank: int,
                          sent_after: list, n_sent: int, wait=None, key_off: int = 0, key_len: int = 10,
                          descending: bool = False) -> torch.Tensor:
    """Receive side of the fine-bucket exchange when every round lands in place: round b's block
    ``rows_in[off[b]:off[b+1]]`` (FineMerge) is ordered into ``rows_out[off[b]:...]``, deferred
    until the send rows under it have gone out (``sent_after``, as in sort_received_rounds).  A
    round whose bucket outgrew LDS is sorted after the last round with local_sort_rows."""
    out = bufs.rows_out
    recv = bufs.recv_rows()
    m = FineMerge(fine, L, fb, B, rank, out, key_off, key_len, descending)
    pending = []
    for b in range(B):
        if wait is not None:
            wait(b)
        pending.append(b)
        keep = []
        for b2 in pending:
            a2, z2 = off[b2], off[b2 + 1]
            if b == B - 1 or z2 <= sent_after[b] or a2 >= n_sent:
                m.merge(b2, recv, a2, a2, z2)
            else:
                keep.append(b2)
        pending = keep
    fl = m.flags.tolist()
    for b in range(B):
        if fl[b]:
            a, z = off[b], off[b + 1]
            ea, eb = _round_scratch(bufs, off[-1], a, z)
            local_sort_rows(recv[a:z], out[a:z], ea, eb, key_off, key_len, descending=descending,
                            hi_bounds=None if descending else fine_hi_bounds(L, fb, rank * B + b))
    return out[: off[-1]]


def _round_scratch(bufs: SortBuffers, n_recv: int, a: int, z: int) -> tuple[torch.Tensor, torch.Tensor]:
    """Two [z - a, 2] int64 entry arrays for re-sorting received rows a..z after the exchange: the
    buffer set's entry arrays when it has 16-byte ones, else the free tail of rows_in past the
    received rows (a pitch-128 set: ~28 bytes per row), else fresh memory."""
    m = z - a
    if bufs.ent_b.numel() >= 2 * z and bufs.ent_a.numel() >= 2 * z:
        return bufs.ent_a.view(-1, 2)[a:z], bufs.ent_b.view(-1, 2)[a:z]
    rec = bufs.rows_out.shape[1]
    flat = bufs.rows_in.view(-1)
    lo = (n_recv * rec + 255) // 256 * 256
    if flat.numel() - lo >= 32 * m:
        t = flat[lo: lo + 32 * m].view(torch.int64).view(2, m, 2)
        return t[0], t[1]
    return (torch.empty((m, 2), dtype=torch.int64, device=flat.device),
            torch.empty((m, 2), dtype=torch.int64, device=flat.device))


def sort_received_rounds(bufs: SortBuffers, off: list, sent_after: list, n_sent: int, seps_hi: list, B: int,
                         rank: int, key_off: int, key_len: int, wait=None, descending: bool = False) -> torch.Tensor:
    """Receive side of the pipelined range shuffle: round b's block ``rows_in[off[b]:off[b+1]]``
    holds all rows of this rank's key range b.  Each is sorted as it arrives (``wait(b)``): E64
    entries of the rows read through LDS with the look-back sort's histograms fused in, the
    look-back radix sort, then the row gather with the run fix-up into ``rows_out[off[b]:...]``,
    deferred until the send rows under it have gone out (``sent_after[b]`` = send rows complete
    after round b; rows past ``n_sent`` never held data).  A look-back failure or a run too long
    for the fix-up is redone after the last round (count + scatter sort, or the full-key sort)."""
    out = bufs.rows_out
    e64a, e64b = bufs.ent_a.view(-1), bufs.ent_b.view(-1)
    compact = S.compact_sort_ok(bufs.rows_in[:2], key_len) and not descending
    flags = torch.zeros((B, 2), dtype=torch.int32, device=out.device)     # [gather overflow, look-back error]
    pending, compact_rounds = [], []
    for b in range(B):
        if wait is not None:
            wait(b)
        a, z = off[b], off[b + 1]
        if z > a:
            hb = _range_hi_bounds(seps_hi, rank * B + b)
            if compact and z - a >= 2:
                r = bufs.rows_in[a:z]
                P = min(S.common_prefix_bits(*hb), 8 * key_len)
                win = min(S.window_bits64(z - a), max(8, ((8 * key_len - P + 7) // 8) * 8), 32)
                e, hist = S.extract_keys64_tile(r, key_off, key_len, P, e64a[a:z], hist=True)
                srt = S.sort_entries64(e, e64b[a:z], win, gen_hist=hist, err=flags[b, 1:])
                pending.append((a, z, b, ("e64", srt, win)))
                compact_rounds.append((a, z, b, P, win))
            else:
                srt = _sort_keys(bufs.rows_in[a:z], bufs.ent_a[a:z], bufs.ent_b[a:z], key_off, key_len, hb,
                                 descending=descending)
                pending.append((a, z, b, ("e128", srt, 0)))
        keep = []
        for a2, z2, b2, (fmt, s2, win) in pending:
            if b == B - 1 or z2 <= sent_after[b] or a2 >= n_sent:
                if fmt == "e64":
                    S.gather_fixup(bufs.rows_in[a2:z2], s2, out[a2:z2], key_off, key_len, win, flags[b2, :1],
                                   err=flags[b2, 1:])
                else:
                    S.gather_rows(bufs.rows_in[a2:z2], entries=s2, out=out[a2:z2])
            else:
                keep.append((a2, z2, b2, (fmt, s2, win)))
        pending = keep
    if compact_rounds:
        fl = flags.tolist()
        for a2, z2, b2, P, win in compact_rounds:
            overflow, failed = fl[b2][0] != 0, fl[b2][1] != 0
            r = bufs.rows_in[a2:z2]
            if failed:        # the look-back sort failed: the entries again, count + scatter passes
                e = S.extract_keys64(r, key_off, key_len, P, e64a[a2:z2])
                srt = S.sort_entries64(e, e64b[a2:z2], win, lookback=False)
                flag = torch.zeros(1, dtype=torch.int32, device=out.device)
                S.gather_fixup(r, srt, out[a2:z2], key_off, key_len, win, flag)
                overflow = int(flag.item()) != 0
            if overflow:      # a run of equal windows too long for the fix-up: full-key sort of the range
                srt = _sort_keys(r, bufs.ent_a[a2:z2], bufs.ent_b[a2:z2], key_off, key_len, None)
                S.gather_rows(r, entries=srt, out=out[a2:z2])
    return out[: off[-1]]

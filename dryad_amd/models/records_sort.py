"""Per-rank program of a multi-rank OrderBy over a COLUMNAR table, on one GPU (loopback).

``bench.py --loopback-ranks W --loopback-table records64`` runs rank ``rank``'s share of

    FromStore(gen://records64 ...).OrderBy(r => r.V1)        (or OrderByDescending, or by r.Key)

on a W-GPU node, as the fused OrderBy of a columnar table runs it (runtime/gpu_executor
._run_fused_columns): the key bounds (the vote carries every rank's), the columns packed into
byte-keyed rows (ops/rowpack: the V1 key part cut to its 31-bit range and recovered from the key
bytes, so a 64-byte record stays a 64-byte row), the fine-bucket send side (E64 window entries,
sample, separators, look-back sort on the top key bits, the send rows packed round by round), the
per-round LDS merge of the received rows, and the unpack into columns.

The all-to-all-v is the only part replaced: the rows this rank receives (round b = the rows of
EVERY source whose key falls in its b-th range, source-major, each source's piece in fine-bucket
order) are built by running every source's pack and bucketing, outside the timed segments; the
other ranks' samples and key bounds likewise.  The rank's input table is generated before the
step (it exists before the job, like an hbm:// input), untimed.

Validated: the output key column is ordered, the output columns' order-independent fingerprint
(utils/validate.py) equals that of the rows received, and the output keys lie in this rank's
fine-bucket range.  Reference: RangePartition + ParallelSort over typed records
(LinqToDryad/DryadLinqVertex.cs:4909-5151, 9330-9335; DryadLinqQueryGen.cs:2362-2474).
"""
from __future__ import annotations

import torch

from ..gpu.table import DeviceTable, Shape
from ..ops import recordsort as RS
from ..ops import relational as R
from ..ops import rowpack as RP
from ..ops import sort as S
from ..ops import terasort as TS
from ..utils import validate as V
from .records_cpu import FIELDS

CHUNK = 1 << 26           # rows per chunk of the untimed simulation passes


class Records64LoopbackJob:
    def __init__(self, W: int, rank: int, n: int, key: str = "V1", descending: bool = False,
                 nkeys: int = 1 << 20, seed: int = 7, device=None, slack: float = 0.01, pack_group: int = 1):
        self.W, self.rank, self.n, self.key, self.desc = W, rank, n, key, descending
        self.nkeys, self.seed, self.pack_group = nkeys, seed, pack_group
        self.dev = dev = torch.device(device or "cuda")
        self.shape = Shape("tuple", list(FIELDS))
        self.cols = [torch.empty(n, dtype=torch.int64, device=dev) for _ in FIELDS]
        R.gen_records64(self.cols, rank * n, nkeys, seed)
        self.table = DeviceTable(n, self.shape, dict(zip(FIELDS, self.cols)))
        m = min(CHUNK, max(n, 1))
        self._scr_cols = [torch.empty(m, dtype=torch.int64, device=dev) for _ in FIELDS]
        per = [RP.key_bounds([self.table.cols[key]], n) if s == rank else self._source_bounds(s) for s in range(W)]
        self.kbounds = RP.merge_bounds(per, 1)
        self.lay = RP.plan(self.table, [self.table.cols[key]], self.kbounds)
        if self.lay is None:
            raise ValueError("records64 loopback: the key does not pack into a sort row")
        rec = self.rec = self.lay.rec
        cap = int(n * (1 + slack)) + 1024
        self.bufs = RS.SortBuffers(rows_in=torch.empty((cap, rec), dtype=torch.uint8, device=dev),
                                   rows_out=torch.empty((cap, rec), dtype=torch.uint8, device=dev),
                                   ent_a=torch.empty(cap, dtype=torch.int64, device=dev),
                                   ent_b=torch.empty(cap, dtype=torch.int64, device=dev))
        self._scr_rows = torch.empty((m, rec), dtype=torch.uint8, device=dev)
        self.B = RS.fine_subs(n * rec, W)
        self.out_cols = None
        self.phases = {}

    @property
    def bytes_per_rank(self) -> int:
        return self.n * 8 * len(FIELDS)

    # ------------------------------------------------------------------ simulated other ranks
    def _source_chunks(self, s: int, packed: bool = True):
        """(first row, chunk table, packed rows) of source s's input, chunk by chunk (untimed)."""
        n = self.n
        for c0 in range(0, n, CHUNK):
            m = min(CHUNK, n - c0)
            cols = [c[:m] for c in self._scr_cols]
            R.gen_records64(cols, s * n + c0, self.nkeys, self.seed)
            t = DeviceTable(m, self.shape, dict(zip(FIELDS, cols)))
            rows = None
            if packed:
                rows = self._scr_rows[:m]
                RP.pack(t, [t.cols[self.key]], self.lay, rows)
            yield c0, t, rows

    def _source_bounds(self, s: int) -> list:
        lo, hi = None, None
        for _, t, _ in self._source_chunks(s, packed=False):
            b = RP.key_bounds([t.cols[self.key]], t.n)
            lo = b[0] if lo is None else min(lo, b[0])
            hi = b[1] if hi is None else max(hi, b[1])
        return [lo, hi]

    def _samples(self, mine: torch.Tensor) -> torch.Tensor:
        """Every rank's sample as the sample all-gather returns it (the others built untimed)."""
        tgt, sseed = 1 << 20, 314159
        m, stride = RS.sample_count(self.n, tgt)
        parts = []
        for s in range(self.W):
            if s == self.rank:
                parts.append(mine)
                continue
            off = RS.sample_offset(sseed, s, stride)
            pos = torch.arange(off, off + stride * m, stride, device=self.dev)[:m]
            got = []
            for c0, t, rows in self._source_chunks(s):
                p = pos[(pos >= c0) & (pos < c0 + t.n)] - c0
                if p.numel():
                    got.append(rows.index_select(0, p))
            sel = torch.cat(got) if got else self._scr_rows[:0]
            e = torch.empty(sel.shape[0], dtype=torch.int64, device=self.dev)
            if sel.shape[0]:
                RS.fine_entries(sel, 0, self.lay.key_len, e, self.desc, hist=False)
            samp = torch.zeros((e.shape[0], 2), dtype=torch.int64, device=self.dev)
            samp[:, 1] = e & RS._WINDOW
            parts.append(samp)
        return torch.cat(parts)

    def _receive(self, L: list, fb: int):
        """The exchange, simulated: every source's rows of this rank's key ranges staged in
        rows_out (dead after the send side), then ordered (round, source, bucket) by one stable
        entry sort and gathered into rows_in, the receive buffer.  Returns (round offsets, fine
        counts [W, K] int32)."""
        W, B, me = self.W, self.B, self.rank
        bufs = self.bufs
        L0, L1 = L[me * B], L[(me + 1) * B]
        K = L1 - L0
        kb = torch.tensor([L[me * B + b] - L0 for b in range(B + 1)], dtype=torch.int64, device=self.dev)
        fine = torch.zeros(W * K, dtype=torch.int64, device=self.dev)
        ent = bufs.ent_a
        pos = 0
        mask = (1 << fb) - 1
        for s in range(W):
            for c0, t, rows in self._source_chunks(s):
                e = torch.empty(t.n, dtype=torch.int64, device=self.dev)
                RS.fine_entries(rows, 0, self.lay.key_len, e, self.desc, hist=False)
                bucket = (e >> (64 - fb)) & mask
                sel = torch.nonzero((bucket >= L0) & (bucket < L1)).view(-1)
                k = sel.numel()
                if k == 0:
                    continue
                if pos + k > bufs.capacity:
                    raise RuntimeError(f"range partition skew: more than {bufs.capacity} rows received")
                bufs.rows_out[pos: pos + k] = rows.index_select(0, sel)
                kk = bucket.index_select(0, sel) - L0
                b = torch.bucketize(kk, kb[1:], right=True)
                comp = (b * W + s) * K + kk
                ent[pos: pos + k] = (comp << 32) | torch.arange(pos, pos + k, dtype=torch.int64, device=self.dev)
                fine += torch.bincount(s * K + kk, minlength=W * K)
                pos += k
        N = pos
        srt = S.sort_entries64(ent[:N], bufs.ent_b[:N], 32, lookback=False)
        TS.pack_rows(bufs.rows_in[:N], bufs.rows_out[:N], srt, N)
        fine = fine.view(W, K)
        per_round = [int(fine[:, int(kb[b]): int(kb[b + 1])].sum()) for b in range(B)]
        off = [0]
        for b in range(B):
            off.append(off[-1] + per_round[b])
        self.recv_src = [[int(fine[s, int(kb[b]): int(kb[b + 1])].sum()) for b in range(B)] for s in range(W)]
        return off, fine.to(torch.int32)

    def _fingerprint_rows(self, rows: torch.Tensor):
        parts = []
        for a in range(0, rows.shape[0], CHUNK):
            r = rows[a: a + CHUNK]
            cols = RP.unpack(r, self.lay)
            parts.append(V.group_fingerprint([cols[f] for f in FIELDS]))
        return V.combine(parts)

    # ------------------------------------------------------------------ the rank's program
    def step(self):
        n, W, B, me = self.n, self.W, self.B, self.rank
        bufs, lay = self.bufs, self.lay
        ev = {k: torch.cuda.Event(enable_timing=True) for k in
              ("t0", "bounds", "pack_cols", "entries", "sample", "plan", "send", "merge0", "merge", "unpack")}
        fb = RS.fine_bits(n * W)
        keyc = self.table.cols[self.key]
        ev["t0"].record()
        RP.key_bounds([keyc], n)                 # (the vote's values; the job's bounds are fixed here)
        ev["bounds"].record()
        RP.pack(self.table, [keyc], lay, bufs.rows_in[:n])
        ev["pack_cols"].record()
        rows = bufs.rows_in[:n]
        e, tmp = bufs.entry_pair(n)
        e, hist = RS.fine_entries(rows, 0, lay.key_len, e, self.desc)
        ev["entries"].record()
        mine = RS.e64_samples(e, n, me, 1 << 20, 314159)
        ev["sample"].record()
        allsamp = self._samples(mine)            # (the sample all-gather: others built untimed)
        sep_ev = torch.cuda.Event(enable_timing=True)
        sep_ev.record()
        seps = RS.separators_from_samples(allsamp, W * B)
        seps_hi = [int(x) & ((1 << 64) - 1) for x in seps[:, 1].tolist()]
        plan = RS.FineSend(bufs, rows, e, tmp, hist, n, seps_hi, B, W, fb, group=self.pack_group,
                           rebuild=lambda: RS.fine_entries(rows, 0, lay.key_len, e, self.desc, hist=False)[0])
        ev["plan"].record()
        pack_ev = [torch.cuda.Event(enable_timing=True) for _ in range(B)]
        for b in range(B):
            plan.pack(b)
            pack_ev[b].record()
        ev["send"].record()
        st, L = plan.st, plan.L
        off, fine = self._receive(L, fb)                          # the all-to-all-v (not timed)
        self.expect_fp = self._fingerprint_rows(bufs.rows_in[: off[-1]])
        ev["merge0"].record()
        recv = bufs.rows_in
        merger = RS.FineMerge(fine, L, fb, B, me, bufs.rows_out, 0, lay.key_len, self.desc)
        merge_ev = [torch.cuda.Event(enable_timing=True) for _ in range(B)]
        for b in range(B):
            merger.merge(b, recv, off[b], off[b], off[b + 1])
            merge_ev[b].record()
        fl = merger.flags.tolist()
        for b in range(B):                   # a bucket past LDS (heavy skew): the round re-sorted
            if fl[b]:
                a, z = off[b], off[b + 1]
                ea = torch.empty((z - a, 2), dtype=torch.int64, device=self.dev)
                RS.local_sort_rows(recv[a:z], bufs.rows_out[a:z], ea, torch.empty_like(ea), 0, lay.key_len,
                                   descending=self.desc)
        ev["merge"].record()
        out_rows = bufs.rows_out[: off[-1]]
        self.out_cols = RP.unpack(out_rows, lay, bufs.rows_in.view(-1))
        ev["unpack"].record()
        torch.cuda.synchronize(self.dev)
        if int(plan.bad.item()):
            raise RuntimeError("send-side pack: an entry named a row past the table")
        el = lambda a, b: a.elapsed_time(b)  # noqa: E731
        self.phases = {"key_bounds_ms": el(ev["t0"], ev["bounds"]), "pack_columns_ms": el(ev["bounds"], ev["pack_cols"]),
                       "entries_ms": el(ev["pack_cols"], ev["entries"]), "sample_ms": el(ev["entries"], ev["sample"]),
                       "separators_entry_sort_ms": el(sep_ev, ev["plan"]), "pack_ms": el(ev["plan"], ev["send"]),
                       "receive_merge_ms": el(ev["merge0"], ev["merge"]), "unpack_ms": el(ev["merge"], ev["unpack"])}
        pk = [el(ev["plan"], pack_ev[0])] + [el(pack_ev[b - 1], pack_ev[b]) for b in range(1, B)]
        mg = [el(ev["merge0"], merge_ev[0])] + [el(merge_ev[b - 1], merge_ev[b]) for b in range(1, B)]
        rec = self.rec
        send_b = [(st[(b + 1) * W] - st[b * W] - (st[b * W + me + 1] - st[b * W + me])) * rec for b in range(B)]
        recv_b = [(off[b + 1] - off[b] - self.recv_src[me][b]) * rec for b in range(B)]
        self.rounds = dict(pack_ms=pk, merge_ms=mg, send_bytes=send_b, recv_bytes=recv_b, st=st, off=off)
        self.L, self.fb = L, fb
        return self.out_cols

    @property
    def ms(self) -> float:
        return sum(self.phases.values())

    def model(self, link_GBps: float) -> dict:
        """MODELLED step with the all-to-all-v on a link of ``link_GBps`` per GPU (as
        TeraSortLoopbackJob.model), the unpack after the last merge.  Labelled modelled."""
        r, ph = self.rounds, self.phases
        t_ready = sum(ph[k] for k in ("key_bounds_ms", "pack_columns_ms", "entries_ms", "sample_ms",
                                      "separators_entry_sort_ms"))
        wire = [max(a, b) / (link_GBps * 1e6) for a, b in zip(r["send_bytes"], r["recv_bytes"])]
        sched = RS.overlap_schedule(r["st"], r["off"], self.B, self.W, r["st"][-1], RS.OVERLAP_SLOTS)
        ov = RS.overlap_model(t_ready, r["pack_ms"], r["merge_ms"], wire, sched, RS.OVERLAP_SLOTS)
        bulk = RS.overlap_model(t_ready, r["pack_ms"], r["merge_ms"], wire, sched, RS.OVERLAP_SLOTS, bulk=True)
        return dict(link_GBps=link_GBps, modelled=True, wire_ms=round(sum(wire), 2),
                    overlapped_step_ms=round(ov["step_ms"] + ph["unpack_ms"], 2),
                    first_round_queued_ms=round(ov["first_queued_ms"], 2), wire_idle_ms=round(ov["wire_idle_ms"], 2),
                    bulk_step_ms=round(bulk["step_ms"] + ph["unpack_ms"], 2))

    def validate(self) -> dict:
        cols = self.out_cols
        k = cols[self.key]
        m = k.shape[0]
        viol = 0
        for a in range(0, max(m - 1, 0), CHUNK):            # adjacent pairs, chunk by chunk
            z = min(m - 1, a + CHUNK)
            lo, hi = k[a:z], k[a + 1: z + 1]
            viol += int(((hi < lo) if not self.desc else (hi > lo)).sum().item())
        got = V.combine([V.group_fingerprint([cols[f][a: a + CHUNK] for f in FIELDS]) for a in range(0, m, CHUNK)])
        in_bounds = True
        if m:
            ends = torch.stack([k[0], k[-1]])
            rows = torch.zeros((2, self.rec), dtype=torch.uint8, device=self.dev)
            t = DeviceTable(2, self.shape, {f: (ends if f == self.key else torch.zeros(2, dtype=torch.int64,
                                                                                        device=self.dev)) for f in FIELDS})
            RP.pack(t, [ends], self.lay, rows)
            e = torch.empty(2, dtype=torch.int64, device=self.dev)
            RS.fine_entries(rows, 0, self.lay.key_len, e, self.desc, hist=False)
            bk = ((e >> (64 - self.fb)) & ((1 << self.fb) - 1)).tolist()
            L0, L1 = self.L[self.rank * self.B], self.L[(self.rank + 1) * self.B]
            in_bounds = all(L0 <= x < L1 for x in bk)
        ok = viol == 0 and got == self.expect_fp and in_bounds
        return dict(ok=bool(ok), order_violations=viol, fingerprint_match=got == self.expect_fp, rows=m,
                    in_bounds=bool(in_bounds))

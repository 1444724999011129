"""TeraSort workload (BASELINE.json headline: "GB/sec sorted (whole node), 1 TB TeraSort").

The DryadLINQ TeraSort experiment (OSDI'08 §5) is a *weak-scaling* sort: every machine holds a
fixed 3.87 GB partition of 100-byte records (10-byte key) and the table grows with the machine
count (240 machines ~ 1 TB).  This module reproduces that job on MI355X ranks: each rank owns
``records_per_rank`` records of the global synthetic table (default 1.25e9 = 125 GB, so 8 ranks
= 1 TB), and one step is

    FromStore(gen) -> OrderBy(r.key) -> ToStore(hbm://)

executed as generate (read the input table) -> sample/range-partition -> RCCL all-to-all-v ->
local radix sort -> row gather into the HBM output table.
"""
from __future__ import annotations

import time
from dataclasses import dataclass

import torch

from ..ops import recordsort as RS
from ..ops import sort as S
from ..ops import terasort as TS
from ..parallel import shuffle
from ..parallel.comm import World, get_world

RECORD = TS.RECORD_BYTES
KEYLEN = TS.KEY_BYTES


@dataclass
class TeraSortConfig:
    records_per_rank: int = 1_250_000_000
    seed: int = 0x5EED_7E4A_50A7
    sample_target: int = 1 << 20
    slack: float = 0.01          # receive-buffer headroom for range-partition skew


class TeraSortJob:
    def __init__(self, cfg: TeraSortConfig, world: World | None = None):
        self.cfg = cfg
        self.world = world or get_world()
        dev = self.world.device
        cap = cfg.records_per_rank if self.world.size == 1 else int(cfg.records_per_rank * (1 + cfg.slack))
        self.bufs = RS.SortBuffers.allocate(cap, RECORD, dev)
        self.n = cfg.records_per_rank
        self.out = None
        self.stats = RS.SortStats()

    @property
    def bytes_per_rank(self) -> int:
        return self.n * RECORD

    def generate(self):
        first = self.world.rank * self.n
        TS.generate(self.bufs.rows_in[: self.n], first, self.cfg.seed)

    def step(self):
        self.generate()
        self.out = RS.distributed_sort_rows(self.bufs, self.n, 0, KEYLEN, self.world,
                                            sample_target=self.cfg.sample_target, stats=self.stats)
        return self.out

    def input_checksum(self) -> tuple[int, int]:
        self.generate()
        acc = TS.check(self.bufs.rows_in[: self.n])
        shuffle.all_reduce_(acc, "sum", self.world)
        return int(acc[0].item()), self.n * self.world.size

    def validate(self, expect_hash: int, expect_records: int) -> dict:
        """valsort: global hash sum, record count, in-rank order and cross-rank boundaries."""
        out = self.out
        acc = TS.check(out)
        cnt = torch.tensor([out.shape[0]], dtype=torch.int64, device=out.device)
        shuffle.all_reduce_(acc, "sum", self.world)
        shuffle.all_reduce_(cnt, "sum", self.world)
        # boundary: last key of rank r <= first key of rank r+1 (empty ranks skipped)
        ends = torch.zeros((1, 2 * KEYLEN + 1), dtype=torch.uint8, device=out.device)
        if out.shape[0] > 0:
            ends[0, 0] = 1
            ends[0, 1:1 + KEYLEN] = out[0, :KEYLEN]
            ends[0, 1 + KEYLEN:] = out[-1, :KEYLEN]
        allends = shuffle.all_gather_tensor(ends, self.world).cpu().numpy()
        boundary_ok = True
        prev_last = None
        for row in allends:
            if row[0] == 0:
                continue
            first, last = bytes(row[1:1 + KEYLEN]), bytes(row[1 + KEYLEN:])
            if prev_last is not None and prev_last > first:
                boundary_ok = False
            prev_last = last
        h = int(acc[0].item())
        ok = (h == expect_hash and int(acc[1].item()) == 0 and int(cnt.item()) == expect_records and boundary_ok)
        return dict(ok=bool(ok), hash_match=h == expect_hash, violations=int(acc[1].item()),
                    records=int(cnt.item()), boundary_ok=boundary_ok)


class TeraSortQueryJob:
    """The same TeraSort expressed as a DryadLINQ query and executed by the GPU executor:

        ctx.FromStore("gen://terasort?...").OrderBy(r => r[0:10]).ToStore("hbm://terasort_out")

    The planner emits Sample -> Separators -> RangePartition -(CrossProduct)-> Merge+Sort; the GPU
    executor recognises the idiom and runs it as one fused gang stage on pooled HBM buffers."""

    OUT = "hbm://terasort_out"

    def __init__(self, cfg: TeraSortConfig, world: World | None = None, gen_fused: bool = False):
        import dryad_amd as D
        self.cfg = cfg
        self.world = world or get_world()
        self.n = cfg.records_per_rank
        W = self.world.size
        self.ctx = D.DryadLinqContext(platform="gpu")
        self.ctx.PartitionCount = W
        self.ctx.ShuffleSlack = cfg.slack
        # default: the input table is materialised (128-byte pitch, as on one GPU) and the
        # fine-bucket exchange reads it; GenFusedShuffle generates the records into the send rows
        self.ctx.GenFusedShuffle = bool(gen_fused)
        # a one-rank RCCL communicator that still exchanges (bench.py --rccl-one-rank): the one
        # partition's OrderBy is planned as the sampled range shuffle of a multi-rank job
        self.ctx.ExchangeOneRank = bool(self.world.force_collectives)
        self.src = f"gen://terasort?records={self.n * W}&partitions={W}&seed={cfg.seed}"
        self.out = None

    @property
    def bytes_per_rank(self) -> int:
        return self.n * RECORD

    def query(self):
        return (self.ctx.FromStore(self.src)
                .OrderBy(lambda r: r[0:10])
                .ToStore(self.OUT, delete_if_exists=True))

    def step(self):
        self.query().SubmitAndWait()
        from ..io.providers import provider_for
        ent = provider_for(self.OUT).get(self.OUT)
        self.out = ent["local"][self.world.rank].rows
        return self.out

    def executor_report(self) -> dict:
        ex = self.ctx._get_executor()
        r = ex.last_result or {}
        return dict(fallbacks=r.get("fallbacks"), timings=r.get("timings"), exchange=r.get("exchange"))

    def input_checksum(self) -> tuple[int, int]:
        rows = torch.empty((self.n, RECORD), dtype=torch.uint8, device=self.world.device)
        TS.generate(rows, self.world.rank * self.n, self.cfg.seed)
        acc = TS.check(rows)
        del rows
        shuffle.all_reduce_(acc, "sum", self.world)
        return int(acc[0].item()), self.n * self.world.size

    validate = TeraSortJob.validate


class TeraSortStoredJob:
    """TeraSort from and to stored tables (the reference's TeraSort reads a partitioned table from
    disk and writes one, DryadLINQ OSDI'08 §5):

        ctx.FromStore("partfile://in").OrderBy(r => r[0:10]).ToStore("partfile://out")

    The input is raw 100-byte rows (partfile ``format: rows``), written once by ``prepare`` from
    the generator (not timed).  A step reads each rank's part through the native chunked reader
    (pinned ring -> HBM, at a 128-byte pitch on one rank), sorts it in HBM and writes the sorted
    part through the native pinned writer (HBM -> pinned ring -> pwrite threads), then commits the
    partfile metadata by rename.  ``report()`` splits the step into read / sort / write."""

    def __init__(self, cfg: TeraSortConfig, world: World | None, src: str, dst: str):
        import dryad_amd as D
        self.cfg = cfg
        self.world = world or get_world()
        self.n = cfg.records_per_rank
        W = self.world.size
        self.ctx = D.DryadLinqContext(platform="gpu")
        self.ctx.PartitionCount = W
        self.ctx.ShuffleSlack = cfg.slack
        # the sorted output: each rank's partition as several part files written at once (one
        # file's page-cache writes serialise on its inode lock, profiles/r4/filewrite_ab2.log)
        self.ctx.PartFileSplitBytes = 2 << 30
        self.prep_ctx = D.DryadLinqContext(platform="gpu")
        self.prep_ctx.PartitionCount = W
        self.src, self.dst = src, dst
        self.gen = f"gen://terasort?records={self.n * W}&partitions={W}&seed={cfg.seed}"
        self.res = None
        self.prepared = None
        self.step_log = []             # per step: seconds, read / write / stage / commit split

    @property
    def bytes_per_rank(self) -> int:
        return self.n * RECORD

    def prepare(self, force: bool = False) -> dict:
        """Write the input table from the generator unless a table of this size is there."""
        from ..io.providers import provider_for
        prov = provider_for(self.src)
        if not force and prov.exists(self.src):
            sch = prov.schema(self.src) or {}
            n, size = prov.stream_info(self.src)
            if sch.get("format") == "rows" and n == self.world.size and size == self.n * RECORD * self.world.size:
                self.prepared = dict(reused=True)
                return self.prepared
        t0 = time.perf_counter()
        self.prep_ctx.FromStore(self.gen).ToStore(self.src, delete_if_exists=True).SubmitAndWait()
        r = self.prep_ctx._get_executor().last_result or {}
        w = r.get("write") or {}
        self.prepared = dict(reused=False, seconds=round(time.perf_counter() - t0, 2),
                             write_GBps=round(w.get("bytes", 0) / 1e9 / max(w.get("seconds", 0), 1e-9), 2))
        return self.prepared

    def step(self):
        t0 = time.perf_counter()
        q = self.ctx.FromStore(self.src).OrderBy(lambda r: r[0:10]).ToStore(self.dst, delete_if_exists=True)
        t1 = time.perf_counter()
        q.SubmitAndWait()
        self.res = dict(self.ctx._get_executor().last_result or {})
        self.res["submit_s"] = dict(build_query=round(t1 - t0, 4), submit_and_wait=round(time.perf_counter() - t1, 4))
        ph = self.res.get("phases") or {}
        self.step_log.append(dict(step_s=round(time.perf_counter() - t0, 4), read_s=(self.res.get("read") or {}).get("seconds"),
                                  write_s=(self.res.get("write") or {}).get("seconds"), stages_s=ph.get("stages"),
                                  commit_s=ph.get("commit")))

    def report(self) -> dict:
        r = self.res or {}
        rd, wr = r.get("read") or {}, r.get("write") or {}
        tm = r.get("timings") or {}
        stage = sum(v for k, v in tm.items() if "OrderBy" in k or "Sort" in k or "Input" in k)
        return dict(read_GB=round(rd.get("bytes", 0) / 1e9, 2), read_s=rd.get("seconds"),
                    read_GBps=round(rd.get("bytes", 0) / 1e9 / max(rd.get("seconds") or 0, 1e-9), 2),
                    write_GB=round(wr.get("bytes", 0) / 1e9, 2), write_s=wr.get("seconds"),
                    write_GBps=round(wr.get("bytes", 0) / 1e9 / max(wr.get("seconds") or 0, 1e-9), 2),
                    # output parts written over the recycled parts of the table the step replaced
                    write_recycled_parts=wr.get("recycled_parts", 0),
                    sort_stage_s_excl_read=round(max(0.0, stage - (rd.get("seconds") or 0)), 3),
                    sort_path=r.get("sort_path"), timings=tm, fallbacks=r.get("fallbacks"),
                    job_phases_s=r.get("phases"), submit_and_wait_s=r.get("submit_s"), steps=self.step_log,
                    prepare=self.prepared)

    input_checksum = TeraSortQueryJob.input_checksum

    def validate(self, expect_hash: int, expect_records: int) -> dict:
        """valsort over the output table streamed back through the chunked reader: rank r checks
        the part files i with i % W == r (hash sum, count, in-part order), the first / last key of
        every part are all-gathered to check the order across parts."""
        from ..io import partfile as PF
        from ..io import reader as RD
        from ..io.providers import parse_uri
        dev, W, me = self.world.device, self.world.size, self.world.rank
        meta = PF.read_meta(parse_uri(self.dst)[1])
        acc = torch.zeros(2, dtype=torch.int64, device=dev)
        ends = torch.zeros((meta.count, 2 * KEYLEN + 1), dtype=torch.uint8, device=dev)
        n_mine, bad_edges = 0, 0
        buf = None
        for i in range(me, meta.count, W):
            path = meta.part_path(i)
            n = meta.parts[i].size // RECORD
            n_mine += n
            step = min(max(n, 1), 1 << 26)
            if buf is None or buf.shape[0] < step:
                buf = torch.empty((step, RECORD), dtype=torch.uint8, device=dev)
            prev = None
            for c0 in range(0, n, step):
                c1 = min(n, c0 + step)
                rows = RD.read_rows_to_device(path, dev, c0 * RECORD, c1 - c0, RECORD, buf)
                TS.check(rows, acc)
                a, b = bytes(rows[0, :KEYLEN].cpu().numpy()), bytes(rows[-1, :KEYLEN].cpu().numpy())
                if c0 == 0:
                    ends[i, 0] = 1
                    ends[i, 1:1 + KEYLEN] = rows[0, :KEYLEN]
                if prev is not None and prev > a:
                    bad_edges += 1
                prev = b
                ends[i, 1 + KEYLEN:] = rows[-1, :KEYLEN]
        del buf
        tot = torch.tensor([int(acc[0].item()), n_mine, int(acc[1].item()) + bad_edges], dtype=torch.int64, device=dev)
        shuffle.all_reduce_(tot, "sum", self.world)
        shuffle.all_reduce_(ends, "sum", self.world)          # every part's row comes from one rank
        boundary_ok, last = True, None
        for row in ends.cpu().numpy():
            if row[0] == 0:
                continue
            if last is not None and last > bytes(row[1:1 + KEYLEN]):
                boundary_ok = False
            last = bytes(row[1 + KEYLEN:])
        h = int(tot[0].item())
        ok = h == expect_hash and int(tot[2].item()) == 0 and int(tot[1].item()) == expect_records and boundary_ok
        return dict(ok=bool(ok), hash_match=h == expect_hash, violations=int(tot[2].item()),
                    records=int(tot[1].item()), boundary_ok=boundary_ok, parts=meta.count)


class TeraSortOOCJob:
    """TeraSort of a partition larger than one GPU sorts in HBM (the 1- and 2-GPU points of the
    1 TB headline): ops/extsort.external_sort in hybrid mode over the generator source.
    The phases work in a quarter of the HBM budget, the range buckets that fit the rest stay sorted
    in HBM, the others go through pinned host DRAM (allocated once per job, like a job's spill
    tier), so only the overflow crosses PCIe.  The output is a ``TieredRows`` table per rank."""

    def __init__(self, cfg: TeraSortConfig, world: World | None = None, budget: int | None = None,
                 descending: bool = False):
        from ..io.hosttable import HostRows
        self.descending = descending
        from ..ops import extsort as EX
        self.EX = EX
        self.cfg = cfg
        self.world = world or get_world()
        self.n = cfg.records_per_rank
        dev = self.world.device
        free, _ = torch.cuda.mem_get_info(dev)
        self.budget = int(budget or free * 0.92)
        # host rows: at most n - (resident room) + one bucket (the suffix stops at a bucket edge)
        W = self.world.size
        work = EX.hybrid_work(self.budget, self.n * RECORD)
        _, cap, _ = EX.plan_geometry(self.n, self.n * W, RECORD, W, work)
        room = self.budget - work - min(256 << 20, self.budget // 16)
        host_rows = max(0, min(int(self.n * (1 + cfg.slack)) + 1024, int(self.n * (1 + cfg.slack)) - room // RECORD + cap))
        self.host = HostRows(max(host_rows, 1), RECORD, 0, KEYLEN)
        self.src = EX.GenTeraSortSource(self.world.rank * self.n, self.n, cfg.seed)
        self.out = None
        self.stats = None

    @property
    def bytes_per_rank(self) -> int:
        return self.n * RECORD

    def step(self):
        st = self.EX.ExtSortStats()
        self.out = None              # the previous output's HBM buckets are this step's to reuse
        self.out = self.EX.external_sort(self.src, 0, KEYLEN, self.world, budget=self.budget, stats=st,
                                         out=self.host, resident=True, descending=self.descending)
        self.stats = st
        return self.out

    def input_checksum(self) -> tuple[int, int]:
        dev = self.world.device
        rows = torch.empty((min(self.n, 1 << 26), RECORD), dtype=torch.uint8, device=dev)
        acc = torch.zeros(2, dtype=torch.int64, device=dev)
        for c0 in range(0, self.n, rows.shape[0]):
            c1 = min(self.n, c0 + rows.shape[0])
            TS.generate(rows[: c1 - c0], self.world.rank * self.n + c0, self.cfg.seed)
            TS.check(rows[: c1 - c0], acc)
        del rows
        shuffle.all_reduce_(acc, "sum", self.world)
        return int(acc[0].item()), self.n * self.world.size

    def validate(self, expect_hash: int, expect_records: int) -> dict:
        m64 = (1 << 64) - 1
        h, bad, first, last = self.EX.check_terasort_host(self.out, descending=self.descending)
        s64 = (h & m64) - (1 << 64) if (h & m64) >= (1 << 63) else (h & m64)
        dev = self.world.device
        tot = torch.tensor([s64, self.out.n, bad], dtype=torch.int64, device=dev)
        shuffle.all_reduce_(tot, "sum", self.world)
        ends = torch.zeros((1, 2 * KEYLEN + 1), dtype=torch.uint8, device=dev)
        if self.out.n:
            ends[0, 0] = 1
            ends[0, 1:1 + KEYLEN] = torch.frombuffer(bytearray(first), dtype=torch.uint8)
            ends[0, 1 + KEYLEN:] = torch.frombuffer(bytearray(last), dtype=torch.uint8)
        allends = shuffle.all_gather_tensor(ends, self.world).cpu().numpy()
        boundary_ok, prev_last = True, None
        for row in allends:
            if row[0] == 0:
                continue
            k0 = bytes(row[1:1 + KEYLEN])
            if prev_last is not None and (prev_last < k0 if self.descending else prev_last > k0):
                boundary_ok = False
            prev_last = bytes(row[1 + KEYLEN:])
        hv = int(tot[0]) & m64
        ok = hv == (expect_hash & m64) and int(tot[2]) == 0 and int(tot[1]) == expect_records and boundary_ok
        return dict(ok=bool(ok), hash_match=hv == (expect_hash & m64), violations=int(tot[2]),
                    records=int(tot[1]), boundary_ok=boundary_ok)

    def report(self) -> dict:
        st = self.stats
        if st is None:
            return {}
        return dict(phases_s={k: round(v, 3) for k, v in st.seconds.items()},
                    pcie_GB={"h2d": round(st.bytes_h2d / 1e9, 1), "d2h": round(st.bytes_d2h / 1e9, 1)},
                    resident_fraction=round(st.resident_rows / max(st.n_out, 1), 3),
                    buckets=st.buckets, resident_buckets=st.resident_buckets, chunks=st.chunks,
                    hbm_budget_gb=round(self.budget / 1e9, 1))


class TeraSortLoopbackJob:
    """The per-rank program of a W-rank TeraSort, run on one GPU (``bench.py --loopback-ranks W``).

    Rank ``rank`` of W ranks owns records [rank * n, (rank + 1) * n) of gen://terasort and does
    exactly what the fused distributed OrderBy does on a node.  By default (``mode`` "table") the
    input is a MATERIALISED table, as the 1-GPU step has it: the generator (or, with ``input_uri``,
    the chunked reader from a partfile://) writes the rank's 125 GB of records at a 128-byte pitch
    with their E64 entries and window histograms, then the fine-bucket send side
    (ops/recordsort.send_fine_rows): the rank's sample, the separators of the W * B key ranges (cut
    to fine-bucket edges), one look-back sort of the entries on the top key bits, the fine-bucket
    starts, ONE gather of the rows into the round-major send buffer.  ``mode`` "gen-fused" runs the
    GenFusedShuffle variant instead (no input table: the records are generated straight into the
    send rows in key order, ``pack_gen_fine``).  Then, per received round, the per-bucket LDS
    merge (ts_tile_merge) into the output table.

    The all-to-all-v is the only part replaced: the bytes this rank would receive (round b = the
    records of EVERY source rank whose key falls in this rank's b-th range, in source order, and
    every source's per-bucket counts) are produced by running each source's send side, outside
    the timed segments.  The other ranks' samples (what the sample all-gather returns) are
    generated outside them too.

    Timed with HIP events: (input) + (sample) + (separators + send side) + (receive-side merge);
    the phases are reported separately.  Validated: the output is in order, holds exactly the
    received records (hash sum and count), and its keys lie inside this rank's separator bounds."""

    def __init__(self, cfg: TeraSortConfig, W: int, rank: int = 0, device=None, mode: str = "table",
                 input_uri: str | None = None, pack_group: int = 1):
        self.cfg, self.W, self.rank = cfg, W, rank
        self.pack_group = pack_group
        self.n = cfg.records_per_rank
        self.dev = torch.device(device or "cuda")
        self.mode = mode
        cap = int(self.n * (1 + cfg.slack))
        self.bufs = RS.SortBuffers.allocate(cap, RECORD, self.dev) if mode == "gen-fused" else \
            RS.SortBuffers.allocate_pitch128(cap, RECORD, self.dev)
        self.B = RS.pipeline_subs(self.n * RECORD, W) if mode == "gen-fused" else RS.fine_subs(self.n * RECORD, W)
        self.input = None if input_uri is None else self._prepare_input(input_uri)
        self.out = None
        self.phases = {}
        self.recv_hash = None
        self.bounds = None

    @property
    def bytes_per_rank(self) -> int:
        return self.n * RECORD

    def _prepare_input(self, uri: str) -> str:
        """partfile:// table of this rank's raw 100-byte rows (one part), written from the
        generator (not timed) unless a part of that size is there.  Returns the part's path."""
        import os
        from ..io import partfile as PF
        from ..io.providers import parse_uri
        from ..io.writer import PartWriter
        scheme, path, _ = parse_uri(uri)
        if scheme not in ("partfile", "file"):
            raise ValueError("--input takes a partfile:// table")
        if PF.exists(path):
            m = PF.read_meta(path)
            if m.count == 1 and m.parts[0].size == self.n * RECORD:
                return m.part_path(0)
        base = PF.default_base(path)
        os.makedirs(os.path.dirname(base), exist_ok=True)
        part = f"{base}.{0:08X}"
        chunk = min(self.n, 1 << 26)
        tmp = torch.empty((chunk, RECORD), dtype=torch.uint8, device=self.dev)
        with PartWriter(part, self.dev) as wr:
            for c0 in range(0, self.n, chunk):
                c1 = min(self.n, c0 + chunk)
                TS.generate(tmp[: c1 - c0], self.rank * self.n + c0, self.cfg.seed)
                wr.write(tmp[: c1 - c0])
        del tmp
        PF.write_meta(path, PF.PartFileMeta(base, [PF.PartEntry(0, self.n * RECORD)]))
        return part

    def _events(self):
        return torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def _receive(self, seps_hi, L, fb):
        """The exchange, simulated: every source's send side run for it (entries, look-back sort,
        fine-bucket starts), its pieces for this rank generated in place, its per-bucket counts
        of this rank's key ranges stacked.  Returns (round offsets, fine counts [W, K])."""
        n, W, B, me, seed = self.n, self.W, self.B, self.rank, self.cfg.seed
        bufs = self.bufs
        # scratch: the entry arrays, or (pitch-128 set) ent_a + the send rows, dead by now
        e = bufs.ent_a.view(-1)[:n]
        tmp = bufs.ent_b.view(-1)[:n] if bufs.ent_b.numel() >= n else bufs.rows_out.view(-1)[: n * 8].view(torch.int64)
        recv = bufs.recv_rows()
        Lt = torch.tensor(L, dtype=torch.int64, device=self.dev)

        def send_side(s):
            TS.gen_entries64(e, s * n, seed, hist=False)
            srt = S.sort_entries64(e, tmp, 8 * ((fb + 7) // 8), lookback=False)
            starts = TS.fine_starts(srt, fb)
            return srt, starts, starts.index_select(0, Lt).tolist()
        sizes, fine = [], []
        for s in range(W):
            _, starts, Sg = send_side(s)
            sizes.append([Sg[me * B + b + 1] - Sg[me * B + b] for b in range(B)])
            fine.append((starts[L[me * B] + 1: L[(me + 1) * B] + 1] - starts[L[me * B]: L[(me + 1) * B]]).clone())
        off = [0]
        for b in range(B):
            off.append(off[-1] + sum(sizes[s][b] for s in range(W)))
        if off[-1] > bufs.capacity:
            raise RuntimeError(f"range partition skew: {off[-1]} rows > capacity {bufs.capacity}")
        for s in range(W):
            srt, _, Sg = send_side(s)
            for b in range(B):
                pos = off[b] + sum(sizes[s2][b] for s2 in range(s))
                g = me * B + b
                if Sg[g + 1] > Sg[g]:
                    TS.gen_gather64(recv[pos: pos + Sg[g + 1] - Sg[g]], srt[Sg[g]: Sg[g + 1]], s * n, seed)
        self.recv_sizes = sizes
        return off, torch.stack(fine)

    def _samples(self, mine):
        """Every rank's sample as the sample all-gather returns it (others generated, untimed)."""
        n, W, me, seed = self.n, self.W, self.rank, self.cfg.seed
        tgt, sseed, M64 = self.cfg.sample_target, 314159, (1 << 64) - 1
        if self.mode == "gen-fused":
            others = [RS.gen_samples((s * n, seed), n, s, s << 32, M64, tgt, sseed, self.dev) for s in range(W) if s != me]
        else:
            others = []
            for s in range(W):
                if s != me:
                    x = RS.gen_samples((s * n, seed), n, s, 0, M64, tgt, sseed, self.dev)
                    x[:, 1] &= RS._as_i64(0xFFFFFFFF00000000)
                    x[:, 0] = 0
                    others.append(x)
        return torch.cat(others[:me] + [mine] + others[me:])

    def step(self):
        n, W, B, me = self.n, self.W, self.B, self.rank
        seed, M64 = self.cfg.seed, (1 << 64) - 1
        dev, bufs = self.dev, self.bufs
        tgt, sseed = self.cfg.sample_target, 314159
        ev = [self._events() for _ in range(4)]
        fb = RS.fine_bits(n * W)
        ev[0][0].record()
        if self.mode == "gen-fused":
            ev[0][1].record()
            mine = RS.gen_samples((me * n, seed), n, me, me << 32, M64, tgt, sseed, dev)
        else:
            e, tmp = bufs.entry_pair(n, in_out=True)
            rows = bufs.rows_in[:n, :RECORD]
            if self.input is None:
                TS.generate_with_keys64_pitch128(bufs.rows_in[:n], me * n, seed, e, None, hist=True)
                hist = S.take_gen_hist(e)
            else:
                from ..io import reader as RD
                RD.read_rows_to_device(self.input, dev, 0, n, RECORD, rows)
                e, hist = S.extract_keys64_tile(bufs.rows_in[:n], 0, KEYLEN, 0, e, hist=True)
            ev[0][1].record()
            mine = RS.e64_samples(e, n, me, tgt, sseed)
        ev[1][0].record()
        ev[1][1].record()
        allsamp = self._samples(mine)
        ev[2][0].record()
        seps = RS.separators_from_samples(allsamp, W * B)
        seps_hi = [int(x) & M64 for x in seps[:, 1].tolist()]
        ev_plan = torch.cuda.Event(enable_timing=True)
        pack_ev = [torch.cuda.Event(enable_timing=True) for _ in range(B)]
        if self.mode == "gen-fused":
            st, pack, counts, L = RS.pack_gen_fine(bufs, (me * n, seed), n, seps_hi, B, W, fb)
            ev_plan.record()
            for b in range(B):
                pack(b)
                pack_ev[b].record()
        else:
            # the send side round by round, as the overlapped exchange packs it (FineSend.pack(b)
            # just before round b's all-to-all-v is queued)
            plan = RS.FineSend(bufs, rows, e, tmp, hist, n, seps_hi, B, W, fb, group=self.pack_group)
            st, counts, L, bad = plan.st, plan.counts, plan.L, plan.bad
            ev_plan.record()
            for b in range(B):
                plan.pack(b)
                pack_ev[b].record()
        ev[2][1].record()
        off, fine = self._receive(seps_hi, L, fb)            # the all-to-all-v (not timed)
        acc = TS.check(bufs.recv_rows()[: off[-1]])
        ev[3][0].record()
        # the receive side round by round (FineMerge, as the exchange merges each received round)
        recv = bufs.recv_rows()
        merger = RS.FineMerge(fine, L, fb, B, me, bufs.rows_out)
        merge_ev = [torch.cuda.Event(enable_timing=True) for _ in range(B)]
        for b in range(B):
            merger.merge(b, recv, off[b], off[b], off[b + 1])
            merge_ev[b].record()
        ev[3][1].record()
        fl = merger.flags.tolist()
        for b in range(B):                   # a bucket past LDS (heavy skew): the round re-sorted
            if fl[b]:
                a, z = off[b], off[b + 1]
                ea, eb = RS._round_scratch(bufs, off[-1], a, z)
                RS.local_sort_rows(recv[a:z], bufs.rows_out[a:z], ea, eb, 0, KEYLEN,
                                   hi_bounds=RS.fine_hi_bounds(L, fb, me * B + b))
        out = bufs.rows_out[: off[-1]]
        torch.cuda.synchronize(dev)
        if self.mode != "gen-fused" and int(bad.item()):
            raise RuntimeError("send-side pack: an entry named a row past the table")
        self.out, self.recv_hash = out, acc
        self.bounds = RS.fine_hi_bounds([L[me * B], L[(me + 1) * B]], fb, 0)
        self.phases = {"input_ms": ev[0][0].elapsed_time(ev[0][1]),
                       "sample_ms": ev[0][1].elapsed_time(ev[1][0]),
                       "separators_entry_sort_ms": ev[2][0].elapsed_time(ev_plan),
                       "pack_ms": ev_plan.elapsed_time(ev[2][1]),
                       "receive_sort_ms": ev[3][0].elapsed_time(ev[3][1])}
        pk = [ev_plan.elapsed_time(pack_ev[0])] + [pack_ev[b - 1].elapsed_time(pack_ev[b]) for b in range(1, B)]
        mg = [ev[3][0].elapsed_time(merge_ev[0])] + [merge_ev[b - 1].elapsed_time(merge_ev[b]) for b in range(1, B)]
        # bytes this rank moves over its links per round (its own slice stays on the GPU)
        send_b = [(st[(b + 1) * W] - st[b * W] - (st[b * W + me + 1] - st[b * W + me])) * RECORD for b in range(B)]
        recv_b = [(off[b + 1] - off[b] - self.recv_sizes[me][b]) * RECORD for b in range(B)]
        self.rounds = dict(pack_ms=pk, merge_ms=mg, send_bytes=send_b, recv_bytes=recv_b, st=st, off=off)
        self.sent_rows = st[-1]
        return out

    def model(self, link_GBps: float) -> dict:
        """MODELLED step of this rank with the all-to-all-v on a link of ``link_GBps`` per GPU (each
        round takes max(bytes out, bytes in) / link): the measured per-round pack and merge times
        of the last step replayed in the overlapped exchange's queue order
        (recordsort._overlapped_fine_exchange, ``overlap_model``), and in the bulk order (every
        round packed before the first goes out).  Labelled modelled: no link is measured here."""
        r, ph = self.rounds, self.phases
        t_ready = ph["input_ms"] + ph["sample_ms"] + ph["separators_entry_sort_ms"]
        wire = [max(a, b) / (link_GBps * 1e6) for a, b in zip(r["send_bytes"], r["recv_bytes"])]
        sched = RS.overlap_schedule(r["st"], r["off"], self.B, self.W, r["st"][-1], RS.OVERLAP_SLOTS)
        ov = RS.overlap_model(t_ready, r["pack_ms"], r["merge_ms"], wire, sched, RS.OVERLAP_SLOTS)
        bulk = RS.overlap_model(t_ready, r["pack_ms"], r["merge_ms"], wire, sched, RS.OVERLAP_SLOTS, bulk=True)
        return dict(link_GBps=link_GBps, modelled=True, wire_ms=round(sum(wire), 2),
                    overlapped_step_ms=round(ov["step_ms"], 2), first_round_queued_ms=round(ov["first_queued_ms"], 2),
                    wire_idle_ms=round(ov["wire_idle_ms"], 2), bulk_step_ms=round(bulk["step_ms"], 2),
                    bulk_first_round_queued_ms=round(bulk["first_queued_ms"], 2))

    @property
    def ms(self) -> float:
        return sum(self.phases.values())

    def validate(self) -> dict:
        out = self.out
        acc = TS.check(out)
        h_in, h_out = int(self.recv_hash[0].item()), int(acc[0].item())
        viol = int(acc[1].item())
        ok_lo = ok_hi = True
        if out.shape[0]:
            first = int.from_bytes(bytes(out[0, :8].cpu().tolist()), "big")
            last = int.from_bytes(bytes(out[-1, :8].cpu().tolist()), "big")
            lo, hi = self.bounds            # hi words of this rank's key ranges (fine-bucket edges)
            ok_lo, ok_hi = first >= lo, last <= hi
        ok = h_in == h_out and viol == 0 and ok_lo and ok_hi
        return dict(ok=bool(ok), hash_match=h_in == h_out, violations=viol, records=int(out.shape[0]),
                    in_bounds=bool(ok_lo and ok_hi))


def run_steps(job, steps: int) -> float:
    """Run ``steps`` steps bracketed by barrier+synchronize; returns max-over-ranks seconds."""
    w = job.world
    dev = w.device
    w.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        job.step()
    torch.cuda.synchronize(dev)
    w.barrier()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    shuffle.all_reduce_(t, "max", w)
    return float(t.item())

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

    def __init__(self, cfg: TeraSortConfig, world: World | None = None):
        import dryad_amd as D
        self.cfg = cfg
        self.world = world or get_world()
        self.n = cfg.records_per_rank
        W = self.world.size
        self.ctx = D.DryadLinqContext(platform="gpu")
        self.ctx.PartitionCount = W
        self.ctx._props["ShuffleSlack"] = cfg.slack
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
        return dict(fallbacks=r.get("fallbacks"), timings=r.get("timings"))

    def input_checksum(self) -> tuple[int, int]:
        rows = torch.empty((self.n, RECORD), dtype=torch.uint8, device=self.world.device)
        TS.generate(rows, self.world.rank * self.n, self.cfg.seed)
        acc = TS.check(rows)
        del rows
        shuffle.all_reduce_(acc, "sum", self.world)
        return int(acc[0].item()), self.n * self.world.size

    validate = TeraSortJob.validate


class TeraSortOOCJob:
    """TeraSort of a partition larger than one GPU sorts in HBM (the 1- and 2-GPU points of the
    1 TB headline): ops/extsort.external_sort in hybrid mode over the generator source.
    The phases work in a quarter of the HBM budget, the range buckets that fit the rest stay sorted
    in HBM, the others go through pinned host DRAM (allocated once per job, like a job's spill
    tier), so only the overflow crosses PCIe.  The output is a ``TieredRows`` table per rank."""

    def __init__(self, cfg: TeraSortConfig, world: World | None = None, budget: int | None = None):
        from ..io.hosttable import HostRows
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
                                         out=self.host, resident=True)
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
        h, bad, first, last = self.EX.check_terasort_host(self.out)
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
            if prev_last is not None and prev_last > bytes(row[1:1 + KEYLEN]):
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

"""Hash join of two 100 GB tables with HBM -> host DRAM spill (BASELINE config "Hash-join two
100 GB tables, spill HBM -> host DRAM").

Tables (gen://records64, 64-byte rows = 8 int64 fields, row store):
  * R  "dimension": keys a bijection of [0, |R|) (mode=dim), payload a function of the key;
  * S  "fact":      keys uniform in [0, |R|), so every S row matches exactly one R row.
Query:  R.Join(S, r => r.Key, s => s.Key, (r, s) => r.V1 + s.V1).Sum()  (plus the match count).

Per rank: both tables are produced in chunks and grace-partitioned (ops/grace.py): rows move to
their rank over xGMI (RCCL all-to-all-v), then straight into per-bucket HBM stores; the buckets
that do not fit the HBM budget spill to pinned host DRAM.  Every bucket pair is then hash joined
on the device (open-addressing table over R's bucket, S streamed through it) with the Sum/Count
of the result selector fused into the probe.  The expected answer is computed from S alone
(validation, outside the timed region).
"""
from __future__ import annotations

import time
from dataclasses import dataclass

import torch

from ..ops import grace as G
from ..ops import relational as R
from ..parallel import shuffle
from ..parallel.comm import World
from .records_cpu import dim_multiplier

SEED_R, SEED_S = 0x5EED_0001, 0x5EED_0002
KH = 0xD1B54A32D192ED03


@dataclass
class HashJoinConfig:
    rows_r: int = 1_562_500_000       # 100 GB of 64-byte rows
    rows_s: int = 1_562_500_000
    chunk_rows: int = 1 << 27         # 8 GB chunks
    hbm_budget: int | None = None
    buckets: int | None = None
    prune: bool = True                # carry only Key + V1 through the grace partitioning
    radix: bool = True                # LDS radix join of the resident buckets


def _i64(v):
    v &= (1 << 64) - 1
    return v - (1 << 64) if v >= (1 << 63) else v


def _lsr(z, s):
    return (z >> s) & ((1 << (64 - s)) - 1)


def mix64_t(z: torch.Tensor) -> torch.Tensor:
    """splitmix64 finaliser on int64 tensors (wrapping arithmetic, logical shifts)."""
    z = z + _i64(0x9E3779B97F4A7C15)
    z = (z ^ _lsr(z, 30)) * _i64(0xBF58476D1CE4E5B9)
    z = (z ^ _lsr(z, 27)) * _i64(0x94D049BB133111EB)
    return z ^ _lsr(z, 31)


class HashJoinJob:
    def __init__(self, world: World, cfg: HashJoinConfig):
        self.w, self.cfg = world, cfg
        W, r = world.size, world.rank
        self.r_lo, self.r_hi = (cfg.rows_r * r) // W, (cfg.rows_r * (r + 1)) // W
        self.s_lo, self.s_hi = (cfg.rows_s * r) // W, (cfg.rows_s * (r + 1)) // W
        self.dim_mult = dim_multiplier(cfg.rows_r)
        self.chunk = torch.empty((cfg.chunk_rows, 8), dtype=torch.int64, device=world.device)
        self.grace = None
        self.last = {}

    def _chunks(self, lo, hi, total=None):
        """Chunk ranges of [lo, hi); with ``total`` every rank yields the same number of chunks
        (possibly empty) because each chunk is a collective exchange."""
        C = self.cfg.chunk_rows
        n = -(-(-(-total // self.w.size)) // C) if total is not None else -(-(hi - lo) // C)
        for j in range(n):
            a = min(hi, lo + j * C)
            yield a, min(hi, a + C)

    def _produce(self, table, a, b):
        rows = self.chunk[: b - a]
        if table == "R":
            R.gen_records64_rows(rows, a, self.cfg.rows_r, SEED_R, self.dim_mult)
        else:
            R.gen_records64_rows(rows, a, self.cfg.rows_r, SEED_S, 0)
        return rows.view(torch.uint8).reshape(b - a, 64)

    def prepare(self):
        """Allocate the bucket stores (HBM or page-locked host) once; reused by every step."""
        cfg = self.cfg
        # per-rank receive estimate: an even share of both tables
        # column pruning: the key selectors read Key and the result selector V1 (bytes 0..15 of
        # both tables), so only those 16 of the 64 bytes travel through the partitioning
        self.grace = G.GraceHashJoin(self.w, 64, 0, 8, {"R": self.r_hi - self.r_lo, "S": self.s_hi - self.s_lo},
                                     cfg.chunk_rows, cfg.hbm_budget, cfg.buckets, build="R",
                                     proj=(0, 16) if cfg.prune else None)

    def release(self):
        if self.grace is not None:
            self.grace.release()
            self.grace = None

    def step(self):
        """One full join (generation = the input read, partition/spill, bucket joins, reduce)."""
        cfg, W = self.cfg, self.w.size
        if self.grace is None:
            self.prepare()
        t0 = time.perf_counter()
        self.grace.reset()
        for t, (lo, hi), tot in (("R", (self.r_lo, self.r_hi), cfg.rows_r), ("S", (self.s_lo, self.s_hi), cfg.rows_s)):
            for a, b in self._chunks(lo, hi, tot):
                self.grace.add_chunk(t, self._produce(t, a, b))
        t1 = time.perf_counter()
        acc = torch.zeros(3, dtype=torch.int64, device=self.w.device)
        # (r, s) => r.V1 + s.V1, then Count/Sum: fused into the probe (V1 = bytes 8..15); all
        # buckets at once through the LDS radix join when they are resident, else bucket by bucket
        if not (cfg.radix and self.grace.join_sum_all("R", "S", 8, 8, acc)):
            for _, lr, rr in self.grace.buckets("R", "S"):
                G.join_sum(lr, rr, 0, 8, 8, 8, acc, self.grace.table, self.grace.log_cap)
        if W > 1:
            shuffle.all_reduce_(acc, "sum", self.w)
        a = acc.tolist()
        res = [a[0], a[1] + a[2]]
        self.last = dict(matches=res[0], sum=res[1], partition_s=t1 - t0, spilled_bytes=self.grace.stats.spilled_bytes,
                         buckets=self.grace.B, in_hbm=self.grace.in_hbm)
        return res

    def expected_pairs(self, first: str = "key") -> tuple[int, int]:
        """(pairs, fingerprint) of the join's output records (first, r.V1, s.V1) from S alone, as
        utils/validate.group_fingerprint hashes them (an order-independent multiset hash): every S
        row meets exactly one R row, whose fields are functions of the key.  ``first``: "key"
        (r.Key) or "v2" (r.V2, the string-key variant's first field)."""
        from ..utils import validate as V
        parts = []
        for a, b in self._chunks(self.s_lo, self.s_hi):
            rows = self._produce("S", a, b).view(torch.int64).reshape(-1, 8)
            key = rows[:, 0]
            f1 = _lsr(mix64_t(_i64(SEED_R + KH) ^ key), 33)
            c0 = key if first == "key" else _lsr(mix64_t(_i64(SEED_R + 2 * KH) ^ key), 33)
            parts.append(V.group_fingerprint([c0, f1, rows[:, 1]]))
        n, fp = V.combine(parts)
        if self.w.size > 1:
            t = torch.tensor([n, _i64(fp)], dtype=torch.int64, device=self.w.device)
            shuffle.all_reduce_(t, "sum", self.w)
            n, fp = int(t[0]), int(t[1]) & ((1 << 64) - 1)
        return n, fp

    def expected(self):
        """(matches, sum) from S alone: every S key hits exactly one R row whose V1 = f(key)."""
        acc = torch.zeros(2, dtype=torch.int64, device=self.w.device)
        for a, b in self._chunks(self.s_lo, self.s_hi):
            rows = self._produce("S", a, b).view(torch.int64).reshape(-1, 8)
            key = rows[:, 0]
            f = _lsr(mix64_t((SEED_R + KH) ^ key), 33)
            acc[0] += key.numel()
            acc[1] += (f + rows[:, 1]).sum()
        if self.w.size > 1:
            shuffle.all_reduce_(acc, "sum", self.w)
        return acc.tolist()

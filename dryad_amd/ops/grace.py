"""Out-of-core (grace) hash join of fixed-width row tables: HBM -> pinned host DRAM spill.

SURVEY §5.7: the reference scales data size by partitioning every stage and spilling sorted
runs to temp files when RAM runs out (DryadLinqVertex.cs:9584-9615); its HashJoin vertex
(DryadLinqVertex.cs:852-897) builds a hash table of the (co-partitioned) inner side.  On a GPU
node the tiers are HBM -> pinned host DRAM (PCIe) -> NVMe, and the join becomes a grace join:

  pass A (per table, streamed in chunks that fit HBM):
     rows chunk -> key entries [HIP extract_keys] -> dest = hash(key) % (W * B) [HIP hash_dest]
       -> stable partition pass on dest [HIP] -> rows gathered into (rank, bucket) order [HIP]
       -> W > 1: RCCL all-to-all-v of the rank ranges (xGMI)
       -> per bucket: device -> pinned host copy on a side stream (spill), overlapping the next
          chunk's compute; or kept in HBM when the whole working set fits the budget
  pass B (per bucket b): both tables' bucket b back to HBM (the next bucket's copies run on the
     side stream while bucket b joins), sort-merge join [HIP radix sort + merge-path ranges]
     and the join's reduction on the device.

Buckets are sized so one bucket pair plus join scratch fits comfortably in HBM.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import torch

from ..parallel import shuffle
from ..parallel.comm import World
from . import relational as R
from . import sort as S


@dataclass
class SpillStats:
    spilled_bytes: int = 0
    buckets: int = 0
    in_hbm: bool = False
    rows: dict = field(default_factory=dict)


class BucketStore:
    """Per-bucket append-only row stores: buckets [0, resident) live in HBM, the rest in
    page-locked host DRAM (hybrid hash join: only what does not fit is spilled)."""

    def __init__(self, nbuckets: int, capacity_rows: int, stride: int, device, resident: int):
        self.B, self.stride = nbuckets, stride
        self.cap = capacity_rows
        self.resident = min(resident, nbuckets)
        self._pinned = []
        self.bufs = []
        for b in range(nbuckets):
            if b < self.resident:
                self.bufs.append(torch.empty((capacity_rows, stride), dtype=torch.uint8, device=device))
            else:
                from ._lib import PinnedHostBuffer
                p = PinnedHostBuffer((capacity_rows, stride))
                self._pinned.append(p)
                self.bufs.append(p.tensor)
        self.fill = [0] * nbuckets

    def on_host(self, b: int) -> bool:
        return b >= self.resident

    def append(self, b: int, rows: torch.Tensor, stream):
        n = rows.shape[0]
        if n == 0:
            return
        f = self.fill[b]
        if f + n > self.cap:
            raise RuntimeError(f"grace bucket {b} overflow ({f + n} > {self.cap} rows): skewed keys")
        if self.on_host(b):
            from ._lib import memcpy_async
            memcpy_async(self.bufs[b][f:f + n], rows, stream)
        else:
            with torch.cuda.stream(stream):
                self.bufs[b][f:f + n].copy_(rows, non_blocking=True)
        self.fill[b] = f + n

    def get(self, b: int):
        return self.bufs[b][: self.fill[b]]

    def reset(self):
        self.fill = [0] * self.B

    def release(self):
        for p in self._pinned:
            p.release()
        self._pinned, self.bufs = [], []


def _partition_rows(rows: torch.Tensor, key_off: int, key_len: int, nparts: int, ent_a, ent_b, out):
    """rows -> rows permuted by hash(key) % nparts (stable) + host list of nparts+1 offsets."""
    n = rows.shape[0]
    e = S.extract_keys(rows, key_off, key_len, 0, out=ent_a[:n])
    R.hash_dest(e, 0, nparts)
    part, starts = S.partition_pass(e, 64, out=ent_b[:n])
    S.gather_rows(rows, entries=part, out=out[:n])
    return out[:n], starts[: nparts + 1].cpu().tolist()


class GraceHashJoin:
    """Grace join of two row tables produced chunk by chunk (``produce(table, chunk_index)``)."""

    def __init__(self, world: World, stride: int, key_off: int, key_len: int, rows_per_rank: dict,
                 chunk_rows: int, hbm_budget: int | None = None, buckets: int | None = None):
        self.w, self.stride, self.key_off, self.key_len = world, stride, key_off, key_len
        dev = world.device
        self.dev = dev
        free = torch.cuda.mem_get_info(dev)[0] if dev.type == "cuda" else 1 << 40
        self.budget = int(hbm_budget if hbm_budget is not None else free * 0.85)
        total = sum(rows_per_rank.values()) * stride
        self.stats = SpillStats()
        scratch_a = chunk_rows * (2 * stride + 40)              # caller's chunk + packed copy + entries
        join_scratch = lambda nbytes: nbytes // stride * 96     # noqa: E731  (sort entries x2, pairs, sums)
        W = world.size
        if total * 1.05 + scratch_a + join_scratch(total) < self.budget:
            nb, resident = 1, 1                                  # everything stays in HBM
        else:
            pair = max(self.budget // 10, 1 << 20)              # one bucket of both tables
            nb = buckets or max(2, -(-int(total * 1.05) // pair))
            nb = min(nb, 256 // W)
            pair_bytes = total * 1.05 / nb
            room = self.budget - scratch_a - 2 * pair_bytes - join_scratch(int(pair_bytes))
            resident = max(0, int(room // pair_bytes))
        self.B = nb
        self.in_hbm = resident >= nb
        self.chunk = chunk_rows
        cap = lambda n: int(n / nb * 1.05) + 65536   # noqa: E731
        self.stores = {t: BucketStore(nb, cap(n), stride, dev, resident) for t, n in rows_per_rank.items()}
        self.stats.buckets, self.stats.in_hbm = nb, self.in_hbm
        self.ent_a = torch.empty((chunk_rows, 2), dtype=torch.int64, device=dev)
        self.ent_b = torch.empty_like(self.ent_a)
        self.pbuf = torch.empty((chunk_rows, stride), dtype=torch.uint8, device=dev)
        self.rbuf = torch.empty((int(chunk_rows * 1.3) + 4096 if world.size > 1 else 0, stride), dtype=torch.uint8,
                                device=dev)
        self.copy_stream = torch.cuda.Stream(dev) if dev.type == "cuda" else None

    def reset(self):
        """Empty every bucket for the next join (host buffers stay allocated and registered:
        page-locking 100 GB costs seconds, so it is done once per job, not per step)."""
        for st in self.stores.values():
            st.reset()
        self.stats = SpillStats(buckets=self.B, in_hbm=self.in_hbm)

    # -------------------------------------------------------------- pass A
    def add_chunk(self, table: str, rows: torch.Tensor):
        W, B = self.w.size, self.B
        if self.copy_stream is not None:
            # pbuf / rbuf are about to be overwritten: wait for the previous chunk's spill copies
            torch.cuda.current_stream(self.dev).wait_stream(self.copy_stream)
        part, st = _partition_rows(rows, self.key_off, self.key_len, W * B, self.ent_a, self.ent_b, self.pbuf)
        if W > 1:
            # dest = rank * B + bucket: rank ranges are contiguous; exchange (rank, bucket) counts
            cnt = torch.tensor([st[i + 1] - st[i] for i in range(W * B)], dtype=torch.int64).view(W, B)
            send_counts = cnt.sum(1).tolist()
            allc = shuffle.all_gather_tensor(cnt.flatten().to(self.w.device), self.w).view(W, W, B).cpu()
            recv_by_src = allc[:, self.w.rank, :]                      # [src, bucket]
            recv_counts = recv_by_src.sum(1).tolist()
            n_recv = sum(recv_counts)
            if n_recv > self.rbuf.shape[0]:
                self.rbuf = torch.empty((int(n_recv * 1.2), self.stride), dtype=torch.uint8, device=self.dev)
            shuffle.alltoallv_bytes(part.reshape(-1), [c * self.stride for c in send_counts],
                                    self.rbuf.reshape(-1), [c * self.stride for c in recv_counts], self.w)
            if self.copy_stream is not None:
                self.copy_stream.wait_stream(torch.cuda.current_stream(self.dev))
            off = 0
            for src in range(W):
                for b in range(B):
                    c = int(recv_by_src[src, b])
                    self.stores[table].append(b, self.rbuf[off:off + c], self.copy_stream)
                    if self.stores[table].on_host(b):
                        self.stats.spilled_bytes += c * self.stride
                    off += c
            moved = n_recv
        else:
            if self.copy_stream is not None:
                self.copy_stream.wait_stream(torch.cuda.current_stream(self.dev))
            for b in range(B):
                self.stores[table].append(b, part[st[b]:st[b + 1]], self.copy_stream)
                if self.stores[table].on_host(b):
                    self.stats.spilled_bytes += (st[b + 1] - st[b]) * self.stride
            moved = part.shape[0]
        self.stats.rows[table] = self.stats.rows.get(table, 0) + moved

    def finish_partitioning(self):
        if self.copy_stream is not None:
            torch.cuda.current_stream(self.dev).wait_stream(self.copy_stream)

    # -------------------------------------------------------------- pass B
    def buckets(self, left: str, right: str):
        """Yield (b, left_rows_b, right_rows_b) in HBM; with spilled stores the next bucket's
        host->device copies overlap the caller's work on the current one."""
        self.finish_partitioning()
        L, Rs = self.stores[left], self.stores[right]
        pending = None
        for b in range(self.B):
            if not L.on_host(b):
                yield b, L.get(b), Rs.get(b)
                continue
            cur = pending if pending is not None else self.stream_in(left, right, b)
            torch.cuda.current_stream(self.dev).wait_stream(self.copy_stream)
            pending = self.stream_in(left, right, b + 1) if b + 1 < self.B else None
            yield b, cur[0], cur[1]

    def stream_in(self, left, right, b):
        out = []
        main = torch.cuda.current_stream(self.dev)
        for t in (left, right):
            h = self.stores[t].get(b)
            d = torch.empty(h.shape, dtype=torch.uint8, device=self.dev)   # allocated on the main stream
            self.copy_stream.wait_stream(main)                             # ... whose earlier work may reuse it
            from ._lib import memcpy_async
            memcpy_async(d, h, self.copy_stream)
            out.append(d)
        return out

    def release(self):
        for st in self.stores.values():
            st.release()


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

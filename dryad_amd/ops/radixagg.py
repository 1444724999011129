"""Radix aggregation: high-cardinality GroupBy on one integer key (csrc/kernels/grace.hip
"Radix aggregation"; K6 of SURVEY §2.3, the reference's hash GroupBy vertices
DryadLinqVertex.cs:437-585).

The sort-based GroupBy orders every row before one segmented reduction reads the value columns
through the row permutation: ~4 radix passes over 8-byte entries plus a random gather of every
value.  Here the rows are hash-partitioned instead, the way the radix join partitions its inputs:

1. pass A reads the key and value COLUMNS once and writes packed 16- or 32-byte rows
   (key, up to three 8-byte values) split by the first digit of the key hash;
2. further digit passes split every partition (``grace.radix_partition``) until a partition holds
   a few hundred distinct keys;
3. one workgroup per partition folds it in an LDS hash table (count + up to three sum / min / max
   accumulators) and appends its groups to the output (chunk reservations, one global atomic per
   16K groups), so the data crosses HBM ~2x per pass and never through a random gather.

The number of digits comes from the sampled distinct-key estimate (~300 distinct keys per
partition; an overestimate only makes partitions smaller).  Partitions whose table fills, or that
hold the table's empty-slot key (INT64_MIN), are folded by a torch fallback.  Group order is
unspecified (LINQ leaves the order of a distributed GroupBy to the partitioning), like the LDS
hash-agg path; integer aggregates are exact and deterministic, float sums are summed by LDS
atomics in arbitrary order.
"""
from __future__ import annotations

import math

import torch

from . import _lib
from ._lib import c_i32, c_u32, c_u64, ptr, stream_of, vp
from . import grace as G

_lib.register_signatures({
    "dr_radix_agg_pack": (c_i32, [vp, vp, c_i32, c_u64, c_u32, c_u64, c_i32, c_i32, vp, vp, vp, vp, vp, vp]),
    "dr_radix_agg_pack_grid": (c_u32, [c_u64, c_u32]),
    "dr_radix_agg_grid": (c_u32, [c_u64]),
    "dr_radix_agg_chunk": (c_u32, []),
    "dr_radix_agg": (c_i32, [vp, c_u32, vp, vp, c_u64, c_u64, c_i32, vp, vp, vp, c_u64, vp, vp, vp, vp, vp, vp,
                             vp]),
})

# When it runs is the job's GroupByAggregation (ops/tuning.py): "auto" only for integer keys whose
# value span is 2^32 or more (there the sort-based GroupBy needs 16-byte entries and is the slower
# one; measured on MI355X, profiles/README.md), "radix" for every large single-integer-key
# GroupBy, "sort" never.
MIN_ROWS = 1 << 22                 # below this the sort-based path is as fast
KEYS_PER_PART = 300                # target distinct keys per final
#                                  partition (LDS table: up to 1024 slots, 3 per row)
MIN_BITS = 11                      # >= 2048 partitions: enough workgroups to fill the chip
MAX_BITS = 24
_OPS = {("sum", 0): 0, ("min", 0): 1, ("max", 0): 2, ("sum", 1): 4, ("min", 1): 5, ("max", 1): 6}
_INT = (torch.int64, torch.int32, torch.int16, torch.int8, torch.uint8, torch.bool)


def distinct_upper_estimate(d: int, m: int, n: int) -> int:
    """Distinct keys of an n-row column from d distinct in an m-row uniform sample: the nd with
    nd (1 - exp(-m / nd)) = d (bisection), or n when the sample is (nearly) all distinct."""
    if m <= 0:
        return n
    if d >= 0.97 * m:
        return n
    lo, hi = float(d), float(n)
    for _ in range(60):
        mid = 0.5 * (lo + hi)
        if mid * (1.0 - math.exp(-m / mid)) < d:
            lo = mid
        else:
            hi = mid
    return int(min(n, max(d, 2.0 * hi)))     # 2x headroom: skew hides keys from a sample


def plan_bits(nd: int) -> list[int]:
    """Digit widths of the passes: ~KEYS_PER_PART distinct keys per final partition, as few passes
    of <= 8 bits as cover them (a pass costs ~2x the rows' bytes of HBM traffic; a narrower digit
    saves less than that)."""
    bits = max(MIN_BITS, min(MAX_BITS, math.ceil(math.log2(max(nd, 1) / KEYS_PER_PART))))
    npass = max(1, math.ceil(bits / 8))
    base, extra = divmod(bits, npass)
    return [base + (1 if i < extra else 0) for i in range(npass)]


def _fallback(rows: torch.Tensor, words: list, accs: list):
    """Fold rows (packed, int64 view [r, w]) with torch: (keys, count, accumulators)."""
    k = rows[:, 0]
    uniq, inv = torch.unique(k, return_inverse=True)
    g = uniq.shape[0]
    cnt = torch.bincount(inv, minlength=g).to(torch.int64)
    outs = []
    for (code, wi) in accs:
        v = rows[:, wi]
        f = code >= 4
        if f:
            v = v.view(torch.float64)
        kind = ("sum", "min", "max")[code & 3]
        if kind == "sum":
            o = torch.zeros(g, dtype=v.dtype, device=v.device).index_add_(0, inv, v)
        else:
            init = (float("inf") if kind == "min" else float("-inf")) if f else \
                (torch.iinfo(torch.int64).max if kind == "min" else torch.iinfo(torch.int64).min)
            o = torch.full((g,), init, dtype=v.dtype, device=v.device).scatter_reduce_(
                0, inv, v, "amin" if kind == "min" else "amax", include_self=True)
        outs.append(o.view(torch.int64) if f else o)
    return uniq, cnt, outs


def _close_holes(total_head: int, tails: list, arrays: list) -> int:
    """Move the groups that sit past the final count into the unused chunk tails below it.
    Returns the number of groups."""
    holes = sorted((int(a), int(b)) for a, b in tails if int(b) > int(a))
    total = total_head - sum(b - a for a, b in holes)
    low = [(a, min(b, total)) for a, b in holes if a < total]
    # data ranges in [total, head) not covered by holes
    data, cur = [], total
    for a, b in holes:
        if b <= cur:
            continue
        if a > cur:
            data.append((cur, a))
        cur = max(cur, b)
    if cur < total_head:
        data.append((cur, total_head))
    if not low:
        return total
    dst, src, i, j, ia, ja = [], [], 0, 0, 0, 0
    while i < len(low) and j < len(data):
        la, lb = low[i]
        da, db = data[j]
        take = min(lb - la - ia, db - da - ja)
        dst.append((la + ia, take))
        src.append((da + ja, take))
        ia += take
        ja += take
        if la + ia == lb:
            i, ia = i + 1, 0
        if da + ja == db:
            j, ja = j + 1, 0
    dev = arrays[0].device
    segs = torch.tensor([[a for a, _ in dst], [a for a, _ in src], [t for _, t in dst]], dtype=torch.int64).to(dev)
    lens = segs[2]
    moved = int(sum(t for _, t in dst))
    seg = torch.repeat_interleave(torch.arange(len(dst), device=dev), lens, output_size=moved)
    first = torch.cumsum(lens, 0) - lens
    within = torch.arange(moved, device=dev) - first[seg]
    di = segs[0][seg] + within
    si = segs[1][seg] + within
    for arr in arrays:
        arr.index_copy_(0, di, arr.index_select(0, si))
    return total


def wide_key(key: torch.Tensor) -> bool:
    """Integer key whose value span does not fit 32 bits (the compact 8-byte sort does not apply)."""
    from . import reduce as RD
    c = key if key.dtype == torch.int64 else key.to(torch.int64)
    mn, mx = RD.reduce_multi(c.shape[0], [(RD.MIN, c, None), (RD.MAX, c, None)], c.device)
    return int(mx) - int(mn) >= (1 << 32)


def wanted(key: torch.Tensor) -> bool:
    """Whether the GroupBy operators route this key through radix_aggregate (GroupByAggregation)."""
    from .tuning import current
    mode = current().groupby_aggregation
    if mode == "sort" or key.shape[0] < MIN_ROWS or key.dtype not in _INT:
        return False
    return mode == "radix" or wide_key(key)


def radix_aggregate(key: torch.Tensor, specs: list, nd_est: int | None = None, force: bool = False):
    """GroupBy on one integer key column.  ``specs``: [(op, vals, dtype)] with op in
    count / sum / min / max (as for relational.seg_reduce_multi).  Returns (keys int64, outs) in
    unspecified group order, or None when the shape does not suit it (more than three distinct
    value columns or accumulators, keys past 2^32 rows, small inputs unless ``force``)."""
    n = key.shape[0]
    if key.dim() != 1 or key.dtype not in _INT or n < 2 or n >= (1 << 32):
        return None
    from .tuning import current
    if not force and (current().groupby_aggregation == "sort" or n < MIN_ROWS):
        return None
    dev = key.device
    k64 = key.to(torch.int64).contiguous()
    cols, accs, where = [], [], []
    for op, vals, dtype in specs:
        if op == "count":
            where.append(("count", None))
            continue
        f = 0 if dtype in _INT else 1
        v = vals.to(torch.float64 if f else torch.int64).contiguous()
        j = next((j for j, c in enumerate(cols) if c.data_ptr() == v.data_ptr() and c.dtype == v.dtype), None)
        if j is None:
            if len(cols) == 3:
                return None
            cols.append(v)
            j = len(cols) - 1
        a = (_OPS[(op, f)], 1 + j)
        if a not in accs:
            if len(accs) == 3:
                return None
            accs.append(a)
        where.append(("acc", accs.index(a)))
    rb = 16 if len(cols) <= 1 else 32
    if nd_est is None:
        from . import relational as R
        d, m = R.estimate_distinct(k64)
        nd_est = distinct_upper_estimate(d, m, n)
    widths = plan_bits(nd_est)
    seed = G.HASH_SEED & (2**64 - 1)
    words = rb // 8
    a_rows = torch.empty((n, words), dtype=torch.int64, device=dev)
    b_rows = torch.empty((n, words), dtype=torch.int64, device=dev) if len(widths) > 1 else None
    # pass A: columns -> packed rows, first digit (the top bits of the hash)
    shift = 64 - widths[0]
    pgrid = int(_lib.lib().dr_radix_agg_pack_grid(c_u64(n), c_u32(rb)))
    counts = G._counts_buf(pgrid << widths[0], dev)
    seg_tile = torch.tensor([0, 0, pgrid], dtype=torch.int64, device=dev)
    ps = torch.empty(1 << widths[0], dtype=torch.int64, device=dev)
    pl = torch.empty(1 << widths[0], dtype=torch.int64, device=dev)
    vptrs = (vp * 3)(*[c.data_ptr() for c in cols] + [0] * (3 - len(cols)))
    _lib.call("dr_radix_agg_pack", ptr(k64), vptrs, len(cols), c_u64(n), c_u32(rb), c_u64(seed), shift,
              widths[0], ptr(seg_tile), ptr(counts), ptr(ps), ptr(pl), ptr(a_rows), stream_of(k64))
    cur, other = a_rows, b_rows
    for w in widths[1:]:
        shift -= w
        ps, pl = G.radix_partition(cur.view(torch.uint8).view(n, rb), other.view(torch.uint8).view(n, rb), ps, pl,
                                   0, 8, shift, w, seed)
        cur, other = other, cur
    nparts = ps.numel()
    del other, a_rows, b_rows          # the ping-pong buffer's memory is reused for the outputs
    grid = int(_lib.lib().dr_radix_agg_grid(c_u64(nparts)))
    chunk = int(_lib.lib().dr_radix_agg_chunk())
    out_cap = n + (grid + 1) * chunk
    okey = torch.empty(out_cap, dtype=torch.int64, device=dev)
    ocnt = torch.empty(out_cap, dtype=torch.int64, device=dev)
    oacc = [torch.empty(out_cap, dtype=torch.int64, device=dev) for _ in accs]
    head = torch.zeros(1, dtype=torch.int64, device=dev)
    ovf_count = torch.zeros(1, dtype=torch.int32, device=dev)
    ovf_list = torch.empty(nparts, dtype=torch.int32, device=dev)
    tails = torch.empty(2 * grid, dtype=torch.int64, device=dev)
    ops = (c_i32 * 3)(*[a[0] for a in accs] + [0] * (3 - len(accs)))
    wds = (c_i32 * 3)(*[a[1] for a in accs] + [0] * (3 - len(accs)))
    optrs = (vp * 3)(*[o.data_ptr() for o in oacc] + [0] * (3 - len(oacc)))
    _lib.call("dr_radix_agg", ptr(cur), c_u32(rb), ptr(ps), ptr(pl), c_u64(nparts), c_u64(seed), len(accs), ops, wds,
              ptr(head), c_u64(out_cap), ptr(okey), ptr(ocnt), optrs, ptr(ovf_count), ptr(ovf_list), ptr(tails),
              stream_of(k64))
    meta = torch.cat([head, ovf_count.to(torch.int64), tails]).tolist()
    head_v, n_ovf, tl = meta[0], meta[1], meta[2:]
    arrays = [okey, ocnt] + oacc
    total = _close_holes(head_v, list(zip(tl[0::2], tl[1::2])), arrays)
    keys, cnt = okey[:total], ocnt[:total]
    acc_out = [o[:total] for o in oacc]
    if n_ovf:
        parts = sorted(ovf_list[:n_ovf].tolist())
        sel = torch.cat([cur[int(ps[p]):int(ps[p]) + int(pl[p])] for p in parts])
        fk, fc, fo = _fallback(sel, [a[1] for a in accs], accs)
        keys, cnt = torch.cat([keys, fk]), torch.cat([cnt, fc])
        acc_out = [torch.cat([a, b]) for a, b in zip(acc_out, fo)]
    del cur
    outs = []
    for kind, i in where:
        if kind == "count":
            outs.append(cnt)
        else:
            o = acc_out[i]
            outs.append(o.view(torch.float64) if accs[i][0] >= 4 else o)
    return keys, outs

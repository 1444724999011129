"""Benchmark validation by group fingerprints.

A GroupBy benchmark that only compares total counts and sums passes a result with groups merged,
split or mislabelled as long as the totals survive.  Here a result is checked group by group
through an order-independent fingerprint: every group's (key, count, sum, min, max) is hashed to
64 bits and the hashes are added (mod 2^64), so the fingerprint does not depend on where the
groups live (partitions, ranks, order) and a single wrong group changes it.  The expected value
comes from an independent path: the input regenerated chunk by chunk, the rows of one key range
at a time sorted by torch and reduced with torch scatter ops (no kernel of this framework on that
path apart from the input generator itself).
"""
from __future__ import annotations

import torch

_C = (-7046029254386353131, -4658895280553007687, 0x2545F4914F6CDD1D, 0x5851F42D4C957F2D,
      0x14057B7EF767814F, 0x27BB2EE687B0B0FD)


def _mix(x: torch.Tensor) -> torch.Tensor:
    x = x ^ (x >> 29)
    x = x * _C[0]
    x = x ^ (x >> 32)
    x = x * _C[1]
    return x ^ (x >> 29)


def group_fingerprint(cols: list) -> tuple[int, int]:
    """(number of groups, fingerprint) of a group table given as int64 columns [key, v1, v2, ...]
    (one row per group, any order)."""
    if not cols or cols[0].numel() == 0:
        return 0, 0
    h = _mix(cols[0].to(torch.int64))
    for j, c in enumerate(cols[1:]):
        h = _mix(h ^ (c.to(torch.int64) * _C[2 + j % 4]))
    s = int(h.sum().item()) & ((1 << 64) - 1)
    return int(cols[0].numel()), s


def combine(parts: list) -> tuple[int, int]:
    """Fingerprints of disjoint group sets (e.g. per rank) -> the fingerprint of their union."""
    return sum(n for n, _ in parts), sum(f for _, f in parts) & ((1 << 64) - 1)


def groups_of(key: torch.Tensor, vals: list, ops: list) -> list:
    """Reference GroupBy by torch ops: sort the keys, one group per distinct key, every value column
    reduced with its op ("count" takes no column, "sum" / "min" / "max").  Returns the group columns
    [key, result per op]."""
    if key.numel() == 0:
        return [key[:0]] + [key[:0] for _ in ops]
    k, order = torch.sort(key.to(torch.int64), stable=True)
    uk, inv, cnt = torch.unique_consecutive(k, return_inverse=True, return_counts=True)
    out = [uk]
    vi = iter(vals)
    for op in ops:
        if op == "count":
            out.append(cnt.to(torch.int64))
            continue
        v = next(vi).to(torch.int64).index_select(0, order)
        if op == "sum":
            r = torch.zeros(uk.numel(), dtype=torch.int64, device=key.device).index_add_(0, inv, v)
        else:
            fill = (1 << 63) - 1 if op == "min" else -(1 << 63)
            r = torch.full((uk.numel(),), fill, dtype=torch.int64, device=key.device)
            r.scatter_reduce_(0, inv, v, reduce="amin" if op == "min" else "amax", include_self=True)
        out.append(r)
    return out


def expected_fingerprint(chunks, ops: list, key_ranges: list, keep=None) -> tuple[int, int]:
    """Fingerprint of the GroupBy of the rows ``chunks()`` yields (a callable returning an iterator
    of [key, value columns...] int64 chunks), one key range [lo, hi) at a time so a range's rows
    fit memory; ``keep(key)`` optionally selects the rows this caller validates (e.g. the keys one
    rank of a hash-partitioned job owns)."""
    parts = []
    for lo, hi in key_ranges:
        ks, vs = [], None
        for cols in chunks():
            m = (cols[0] >= lo) & (cols[0] < hi)
            if keep is not None:
                m &= keep(cols[0])
            ks.append(cols[0][m])
            if vs is None:
                vs = [[] for _ in cols[1:]]
            for j, c in enumerate(cols[1:]):
                vs[j].append(c[m])
        if not ks:
            continue
        key = torch.cat(ks)
        vals = [torch.cat(v) for v in (vs or [])]
        parts.append(group_fingerprint(groups_of(key, vals, ops)))
    return combine(parts)


def key_ranges(key_lo: int, key_hi: int, pieces: int) -> list:
    """[lo, hi) ranges splitting the key span [key_lo, key_hi] into ``pieces``."""
    span = key_hi - key_lo + 1
    step = -(-span // max(1, pieces))
    return [(key_lo + i * step, min(key_hi + 1, key_lo + (i + 1) * step)) for i in range(pieces)
            if key_lo + i * step <= key_hi]

"""Python wrappers of the relational HIP kernels (csrc/kernels/relational.hip)."""
from __future__ import annotations

import ctypes
import os

import torch

from . import _lib
from ._lib import c_i32, c_i64, c_u32, c_u64, ptr, stream_of, vp

_lib.register_signatures({
    "dr_build_keys": (c_i32, [ctypes.POINTER(vp), ctypes.POINTER(c_i32), ctypes.POINTER(c_i32), c_i32, c_u64, c_u32,
                              vp, ctypes.POINTER(c_i32), vp]),
    "dr_hash_dest": (c_i32, [vp, c_u64, c_u64, c_u32, vp]),
    "dr_segment_flags": (c_i32, [vp, c_u64, c_u64, vp, vp]),
    "dr_seg_reduce": (c_i32, [vp, vp, vp, c_u64, vp, c_i32, c_i32, vp]),
    "dr_join_ranges": (c_i32, [vp, c_u64, vp, c_u64, c_u64, vp, vp, vp]),
    "dr_join_emit": (c_i32, [vp, vp, c_u64, vp, vp, vp, vp, vp, vp]),
    "dr_scan_i64_workspace": (c_u64, [c_u64]),
    "dr_scan_i64": (c_i32, [vp, vp, c_u64, vp, vp]),
})

KEY_TYPES = {torch.uint8: 0, torch.int8: 1, torch.bool: 2, torch.int16: 3, torch.uint16: 4, torch.int32: 5,
             torch.uint32: 6, torch.int64: 7, torch.uint64: 8, torch.float32: 9, torch.float64: 10}
KEY_BITS = {0: 8, 1: 8, 2: 8, 3: 16, 4: 16, 5: 32, 6: 32, 7: 64, 8: 64, 9: 32, 10: 64}

OP_SUM, OP_MIN, OP_MAX, OP_COUNT = 0, 1, 2, 3


def key_bit_count(cols) -> int:
    return sum(KEY_BITS[KEY_TYPES[c.dtype]] for c in cols)


def build_keys(cols: list, descending=None, idx_base: int = 0, out: torch.Tensor | None = None):
    """Typed key columns (<= 96 bits total) -> (E128 entries [n,2] int64, begin_bit, lo_mask)."""
    n = cols[0].shape[0]
    if n + idx_base >= (1 << 32):
        raise ValueError("build_keys: row index does not fit the 32-bit index field")
    dev = cols[0].device
    if out is None:
        out = torch.empty((n, 2), dtype=torch.int64, device=dev)
    cols = [c.contiguous() for c in cols]
    arr = (vp * len(cols))(*[c.data_ptr() for c in cols])
    ty = (c_i32 * len(cols))(*[KEY_TYPES[c.dtype] for c in cols])
    de = (c_i32 * len(cols))(*[int(bool(d)) for d in (descending or [False] * len(cols))])
    bb = c_i32(0)
    _lib.call("dr_build_keys", arr, ty, de, len(cols), c_u64(n), c_u32(idx_base), ptr(out), ctypes.byref(bb),
              stream_of(out))
    bits = key_bit_count(cols)
    # lo bits that hold key material (everything above the 32-bit row index)
    key_lo_bits = max(0, bits - 64)
    lo_mask = (((1 << key_lo_bits) - 1) << (64 - key_lo_bits)) if key_lo_bits else 0
    return out[:n], bb.value, lo_mask


def hash_dest(entries: torch.Tensor, lo_mask: int, nparts: int) -> torch.Tensor:
    """Internal bucket hash (grace join buckets; both join sides use it).  Not the partitioner
    hash: keyed shuffles use stable_hash_dest, which matches the host path."""
    if not 0 < nparts <= 256:
        raise ValueError(f"hash_dest: {nparts} buckets (1..256)")
    _lib.call("dr_hash_dest", ptr(entries), c_u64(entries.shape[0]), c_u64(lo_mask & (2**64 - 1)), c_u32(nparts),
              stream_of(entries))
    return entries


def segment_flags(entries: torch.Tensor, lo_mask: int) -> torch.Tensor:
    n = entries.shape[0]
    flags = torch.empty(n, dtype=torch.int64, device=entries.device)
    _lib.call("dr_segment_flags", ptr(entries), c_u64(n), c_u64(lo_mask & (2**64 - 1)), ptr(flags), stream_of(entries))
    return flags


def scan_exclusive(a: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    assert a.dtype == torch.int64 and a.is_contiguous()
    n = a.shape[0]
    if out is None:
        out = torch.empty_like(a)
    ws = torch.empty(int(_lib.lib().dr_scan_i64_workspace(c_u64(max(n, 1)))), dtype=torch.uint8, device=a.device)
    _lib.call("dr_scan_i64", ptr(a), ptr(out), c_u64(n), ptr(ws), stream_of(a))
    return out


_lib.register_signatures({"dr_segment_ids": (c_i32, [vp, c_u64, c_u64, vp, vp, vp, vp])})


def segment_ids(entries: torch.Tensor, lo_mask: int):
    """(segment id per sorted row, number of segments, segment start positions): two fused passes
    over the sorted entries (dr_segment_ids), no flag array."""
    n = entries.shape[0]
    dev = entries.device
    ids = torch.empty(n, dtype=torch.int64, device=dev)
    if n == 0:
        return ids, 0, ids
    starts = torch.empty(n, dtype=torch.int64, device=dev)
    ws = torch.empty(int(_lib.lib().dr_scan_i64_workspace(c_u64(n))), dtype=torch.uint8, device=dev)
    _lib.call("dr_segment_ids", ptr(entries), c_u64(n), c_u64(lo_mask & (2**64 - 1)), ptr(ids), ptr(starts), ptr(ws),
              stream_of(entries))
    nseg = int(ids[-1].item()) + 1
    starts = starts[:nseg]
    if nseg * 2 < n:
        starts = starts.clone()      # release the n-row buffer
    return ids, nseg, starts


def _ids_from_flags(flags: torch.Tensor):
    ids = scan_exclusive(flags)
    n = flags.shape[0]
    if n == 0:
        return ids, 0, ids
    nseg = int(ids[-1].item() + flags[-1].item())
    # ids are exclusive sums: segment id of row i = (#starts before i) + flag[i] - 1
    ids = ids + flags - 1
    starts = torch.nonzero(flags, as_tuple=False).flatten()
    return ids, nseg, starts


def seg_reduce(vals: torch.Tensor | None, entries: torch.Tensor | None, seg: torch.Tensor, nseg: int, op: int,
               dtype: torch.dtype = torch.float64) -> torch.Tensor:
    """Segmented reduction over rows in sorted order (row = entries[i].lo & 0xffffffff)."""
    n = seg.shape[0]
    dev = seg.device
    dt = 0 if dtype in (torch.int64, torch.int32, torch.int16, torch.int8, torch.uint8, torch.bool) else 1
    tdt = torch.int64 if dt == 0 else torch.float64
    if op == OP_MIN:
        init = torch.iinfo(torch.int64).max if dt == 0 else float("inf")
    elif op == OP_MAX:
        init = torch.iinfo(torch.int64).min if dt == 0 else float("-inf")
    else:
        init = 0
    out = torch.full((nseg,), init, dtype=tdt, device=dev)
    v = None
    if op != OP_COUNT:
        v = vals.to(tdt).contiguous()
    _lib.call("dr_seg_reduce", ptr(v), ptr(entries), ptr(seg), c_u64(n), ptr(out), op, dt, stream_of(seg))
    return out


_lib.register_signatures({
    "dr_hj_slots": (c_i32, [vp, c_u64, c_u64, c_i32, vp, vp, vp]),
    "dr_hj_gather": (c_i32, [vp, c_u64, vp, vp, vp]),
    "dr_hj_probe": (c_i32, [vp, c_u64, vp, vp, c_i32, c_u64, vp, vp, vp, vp, c_i32, vp]),
})


def hash_join_pairs(outer: torch.Tensor, inner: torch.Tensor, lo_mask: int):
    """Row-index pairs (outer_row, inner_row) of equal keys through a device hash table built on
    the inner entries (csrc/kernels/hashjoin.hip).  Pairs come in outer row order and, per outer
    row, in inner row order (LINQ Join order); ``count[o]`` = matches of outer row o.  Entries must
    be in row order (row index = position), as build_keys / extract_keys produce them."""
    from . import sort as S
    no, ni = outer.shape[0], inner.shape[0]
    dev = outer.device
    lm = c_u64(lo_mask & (2**64 - 1))
    log_cap = max(1, (2 * max(ni, 1) - 1).bit_length())
    slots = torch.empty((ni, 2), dtype=torch.int64, device=dev)
    hist = torch.zeros((1 << log_cap) + 1, dtype=torch.int64, device=dev)
    st = stream_of(hist)
    _lib.call("dr_hj_slots", ptr(inner), c_u64(ni), lm, log_cap, ptr(slots), ptr(hist), st)
    srt = S.sort_entries(slots, 64, 64 + 8 * ((log_cap + 7) // 8)) if ni else slots
    starts = scan_exclusive(hist)
    keys = torch.empty((ni, 2), dtype=torch.int64, device=dev)
    _lib.call("dr_hj_gather", ptr(srt), c_u64(ni), ptr(inner), ptr(keys), st)
    count = torch.empty(no, dtype=torch.int64, device=dev)
    _lib.call("dr_hj_probe", ptr(outer), c_u64(no), ptr(keys), ptr(starts), log_cap, lm, ptr(count), None, None,
              None, 0, st)
    if no == 0:
        z = torch.empty(0, dtype=torch.int64, device=dev)
        return z, z, count
    offs = scan_exclusive(count)
    total = int((offs[-1] + count[-1]).item())
    oo = torch.empty(total, dtype=torch.int64, device=dev)
    ii = torch.empty(total, dtype=torch.int64, device=dev)
    if total:
        _lib.call("dr_hj_probe", ptr(outer), c_u64(no), ptr(keys), ptr(starts), log_cap, lm, None, ptr(offs),
                  ptr(oo), ptr(ii), 1, st)
    return oo, ii, count


def merge_join_pairs(outer_sorted: torch.Tensor, inner_sorted: torch.Tensor, lo_mask: int):
    """Row-index pairs (outer_row, inner_row) of equal keys between two sorted entry arrays,
    grouped by outer in sorted-key order."""
    no, ni = outer_sorted.shape[0], inner_sorted.shape[0]
    dev = outer_sorted.device
    lower = torch.empty(no, dtype=torch.int64, device=dev)
    count = torch.empty(no, dtype=torch.int64, device=dev)
    _lib.call("dr_join_ranges", ptr(outer_sorted), c_u64(no), ptr(inner_sorted), c_u64(ni),
              c_u64(lo_mask & (2**64 - 1)), ptr(lower), ptr(count), stream_of(outer_sorted))
    offs = scan_exclusive(count)
    total = int((offs[-1] + count[-1]).item()) if no else 0
    oo = torch.empty(total, dtype=torch.int64, device=dev)
    ii = torch.empty(total, dtype=torch.int64, device=dev)
    _lib.call("dr_join_emit", ptr(outer_sorted), ptr(inner_sorted), c_u64(no), ptr(lower), ptr(count), ptr(offs),
              ptr(oo), ptr(ii), stream_of(outer_sorted))
    return oo, ii, count


_lib.register_signatures({"dr_gen_records64": (c_i32, [vp, c_i32, c_u64, c_u64, c_u64, c_u64, c_u64, vp]),
                          "dr_gen_records64_rows": (c_i32, [vp, c_i32, c_u64, c_u64, c_u64, c_u64, c_u64, vp])})


def gen_records64_rows(out: torch.Tensor, first: int, nkeys: int, seed: int, dim_mult: int = 0):
    """Row-major gen://records64: ``out`` int64 [n, ncols] (a [n, 64]-byte row store for 8 columns)."""
    _lib.require_gpu_tensor(out, "gen_records64_rows")
    assert out.dtype == torch.int64 and out.dim() == 2
    _lib.call("dr_gen_records64_rows", ptr(out), out.shape[1], c_u64(out.shape[0]), c_u64(first), c_u64(nkeys),
              c_u64(seed & (2**64 - 1)), c_u64(dim_mult), stream_of(out))
    _lib.written(out)
    return out


def gen_records64(cols: list, first: int, nkeys: int, seed: int, dim_mult: int = 0):
    """Fill int64 HBM columns (Key, V1..) with records first.. of gen://records64
    (``dim_mult`` != 0: dimension-table mode, key = (i * dim_mult + seed) % nkeys)."""
    n = cols[0].shape[0]
    for c in cols:
        _lib.require_gpu_tensor(c, "gen_records64")
        assert c.dtype == torch.int64 and c.shape[0] == n
    ptrs = torch.tensor([c.data_ptr() for c in cols], dtype=torch.int64, device=cols[0].device)
    _lib.call("dr_gen_records64", ptr(ptrs), len(cols), c_u64(n), c_u64(first), c_u64(nkeys),
              c_u64(seed & (2**64 - 1)), c_u64(dim_mult), stream_of(cols[0]))
    _lib.written(*cols)
    return cols


_lib.register_signatures({"dr_seg_reduce_multi": (c_i32, [vp, vp, c_u64, c_i32, vp, vp, vp, vp, vp]),
                          "dr_group_chunk_elems": (c_u32, []),
                          "dr_group_chunk_starts": (c_i32, [vp, c_u64, vp, vp]),
                          "dr_seg_reduce_multi_keys": (c_i32, [vp, c_u64, vp, c_u64, vp, c_i32, vp, vp, vp, vp, vp])})

_MOPS = {("sum", 0): 0, ("min", 0): 1, ("max", 0): 2, ("count", 0): 3, ("sum", 1): 4, ("min", 1): 5, ("max", 1): 6}
# value columns of a permuted segmented reduction over at least this many rows are first packed
# into 32- / 40-byte rows (dr_pack_wide) so each sorted entry costs one sector-aligned random read
# instead of one cache line per column: GroupBy of 1.25e9 rows x 3 columns 249.4 -> 238.7 ms per
# step (the torch.stack packing tried first cost 47 ms and lost; profiles/README.md)
AOS_MIN_ROWS = 1 << 24


FUSED_GROUP_KEYS = True


def group_reduce_sorted(srt: torch.Tensor, specs: list, key_xor: int):
    """GroupBy over entries sorted by one 64-bit key word (``int_key_sort`` layout: lo = row, hi =
    normalised key) without materialising segment ids: a chunk pass counts the group starts per
    512 entries, and the multi-aggregate reduction derives every element's group from key changes
    and writes each group's key (hi ^ key_xor) itself.  Returns (keys int64 [nseg], outs)."""
    n = srt.shape[0]
    dev = srt.device
    ch = int(_lib.lib().dr_group_chunk_elems())
    cnt = torch.empty(-(-n // ch), dtype=torch.int64, device=dev)
    _lib.call("dr_group_chunk_starts", ptr(srt), c_u64(n), ptr(cnt), stream_of(srt))
    base = scan_exclusive(cnt)
    nseg = int((base[-1] + cnt[-1]).item())
    keys = torch.empty(nseg, dtype=torch.int64, device=dev)
    outs = seg_reduce_multi(srt, None, nseg, specs, fused=(base, key_xor, keys))
    return keys, outs


def seg_reduce_multi(entries: torch.Tensor | None, seg: torch.Tensor | None, nseg: int, specs: list,
                     fused: tuple | None = None) -> list:
    """Several segmented reductions in ONE pass over the sorted entries.

    ``specs``: [(op, vals, dtype)] with op in sum/min/max/count, vals a column in original row
    order (None for count) and dtype torch.int64 or torch.float64.  Returns one [nseg] tensor per
    spec.  With a row permutation (``entries``), several value columns and many rows, the columns
    are packed into one row-major buffer first (the kernel reads strided values).  ``fused =
    (chunk_base, key_xor, keys_out)``: no ``seg`` array (group_reduce_sorted)."""
    n = entries.shape[0] if fused is not None else seg.shape[0]
    dev = entries.device if fused is not None else seg.device
    outs, keep = [], []
    ops = (ctypes.c_int * max(1, len(specs)))()
    vps = (ctypes.c_void_p * max(1, len(specs)))()
    ops_p = (ctypes.c_void_p * max(1, len(specs)))()
    strides = (ctypes.c_uint32 * max(1, len(specs)))(*([1] * max(1, len(specs))))
    for a, (op, vals, dtype) in enumerate(specs):
        f = 0 if dtype in (torch.int64, torch.int32, torch.int16, torch.int8, torch.uint8, torch.bool) else 1
        tdt = torch.int64 if f == 0 else torch.float64
        if op == "count":
            f, tdt = 0, torch.int64
        init = {"sum": 0, "count": 0,
                "min": torch.iinfo(torch.int64).max if f == 0 else float("inf"),
                "max": torch.iinfo(torch.int64).min if f == 0 else float("-inf")}[op]
        out = torch.full((nseg,), init, dtype=tdt, device=dev)
        outs.append(out)
        ops[a] = _MOPS[(op, f)]
        ops_p[a] = out.data_ptr()
        if isinstance(vals, StridedCol) and op != "count":
            keep.append(None)      # already in the reduced dtype, inside a row-major buffer
            vps[a] = vals.base.data_ptr() + 8 * vals.word
            strides[a] = vals.stride
            continue
        v = None if op == "count" else vals.to(tdt).contiguous()
        keep.append(v)
        vps[a] = v.data_ptr() if v is not None else 0
    cols = [a for a, v in enumerate(keep) if v is not None]
    distinct = list({keep[a].data_ptr(): keep[a] for a in cols}.values())
    if entries is not None and n >= AOS_MIN_ROWS and 2 <= len(distinct) <= 4:
        # one streaming pass packs the distinct columns into 32- / 40-byte rows (the wide sort
        # entry layout with no key: words lo, p0, p1[, p2]), so each permuted row costs one
        # sector-aligned read instead of one cache line per column
        words = 4 if len(distinct) <= 3 else 5
        aos = torch.empty((n, words), dtype=torch.int64, device=dev)
        vp4 = [c.data_ptr() for c in distinct] + [0] * (4 - len(distinct))
        _lib.call("dr_pack_wide", words, vp(0), c_i64(0), *[vp(x) for x in vp4], c_u64(n), ptr(aos), stream_of(aos))
        keep.append(aos)
        slot = {c.data_ptr(): _PAYLOAD_WORDS[j] for j, c in enumerate(distinct)}
        for a in cols:
            vps[a] = aos.data_ptr() + 8 * slot[keep[a].data_ptr()]
            strides[a] = words
    if n and specs:
        for k in range(0, len(specs), 8):     # kernel takes 8 aggregates per pass
            m = min(8, len(specs) - k)
            o8 = (ctypes.c_int * m)(*[ops[k + j] for j in range(m)])
            v8 = (ctypes.c_void_p * m)(*[vps[k + j] for j in range(m)])
            p8 = (ctypes.c_void_p * m)(*[ops_p[k + j] for j in range(m)])
            s8 = (ctypes.c_uint32 * m)(*[strides[k + j] for j in range(m)])
            if fused is not None:
                base, kx, keys_out = fused
                _lib.call("dr_seg_reduce_multi_keys", ptr(entries), c_u64(n), ptr(base),
                          c_u64(kx & (2**64 - 1)), ptr(keys_out), m, o8, v8, p8, s8, stream_of(entries))
            else:
                _lib.call("dr_seg_reduce_multi", ptr(entries), ptr(seg), c_u64(n), m, o8, v8, p8, s8,
                          stream_of(seg))
    return outs


class StridedCol:
    """A 64-bit column stored as word ``word`` of every ``stride``-word row of ``base``."""

    def __init__(self, base: torch.Tensor, word: int, stride: int):
        self.base, self.word, self.stride = base, word, stride


_lib.register_signatures({
    "dr_pack_wide": (c_i32, [c_i32, vp, c_i64, vp, vp, vp, vp, c_u64, vp, vp]),
    "dr_hi_flags": (c_i32, [vp, c_u32, c_u64, vp, vp]),
    "dr_sort_wide": (c_i32, [c_i32, vp, vp, c_u64, c_i32, c_i32, vp, vp, ctypes.POINTER(c_i32)]),
    "dr_sort_u256_workspace": (c_u64, [c_u64]),
})

# payload sort: GroupBy on one int64 key folding <= 4 value columns, on at least this many rows
# and keys spanning <= 32 varying bits (4 radix passes).  Off by default: on the 1.25e9-row
# GroupBy benchmark it measured 260.6 ms against 251.2 ms for the key-pointer sort — the E256
# scatter passes (26 ms each vs 12 for E128) and their count passes cost more than the random
# gathers they remove (profiles/README.md)
PAYLOAD_SORT_MIN_ROWS = 1 << 62
PAYLOAD_SORT_MAX_PASSES = 4
_PAYLOAD_WORDS = (0, 2, 3, 4)      # payload words of an E256 / E320 entry: lo, p0, p1, p2 (hi = key)


def payload_groups(key: torch.Tensor, specs: list):
    """Sort-based GroupBy that carries the aggregated values in the sort entries (32-byte E256:
    key - min(key) in hi, up to three 8-byte values in lo / p0 / p1, or a 40-byte E320 with a
    fourth in p2; csrc/kernels/sort.hip dr_sort_wide),
    then one sequential segmented reduction over the sorted array — no random gather through a
    row permutation.  ``specs`` as for seg_reduce_multi.  Returns (keys, outs) in ascending key
    order (the order of the key-pointer path), or None when the shape does not suit it."""
    from . import reduce as RD
    n = key.shape[0]
    dev = key.device
    if key.dtype != torch.int64 or key.dim() != 1 or n < 2 or n >= (1 << 32):
        return None
    cols, where = [], []
    for op, vals, dtype in specs:
        if op == "count":
            where.append(None)
            continue
        f = dtype not in (torch.int64, torch.int32, torch.int16, torch.int8, torch.uint8, torch.bool)
        v = vals.to(torch.float64 if f else torch.int64).contiguous()
        j = next((j for j, c in enumerate(cols) if c.data_ptr() == v.data_ptr() and c.dtype == v.dtype), None)
        if j is None:
            if len(cols) == 4:
                return None
            cols.append(v)
            j = len(cols) - 1
        where.append(j)
    mn, mx = RD.reduce_multi(n, [(RD.MIN, key, None), (RD.MAX, key, None)], dev)
    span = (mx - mn).bit_length()      # entries hold key - min (order-preserving, >= 0)
    passes = (span + 7) // 8
    if passes > PAYLOAD_SORT_MAX_PASSES:
        return None
    k = key.contiguous()
    words = 4 if len(cols) <= 3 else 5
    e = torch.empty((n, words), dtype=torch.int64, device=dev)
    vp4 = [c.data_ptr() for c in cols] + [0] * (4 - len(cols))
    _lib.call("dr_pack_wide", words, ptr(k), c_i64(mn), *[vp(x) for x in vp4], c_u64(n), ptr(e), stream_of(e))
    del cols
    if passes:
        tmp = torch.empty_like(e)
        ws = torch.empty(int(_lib.lib().dr_sort_u256_workspace(c_u64(n))), dtype=torch.uint8, device=dev)
        flag = ctypes.c_int32(0)
        _lib.call("dr_sort_wide", words, ptr(e), ptr(tmp), c_u64(n), 64, 64 + 8 * passes, ptr(ws), stream_of(e),
                  ctypes.byref(flag))
        if flag.value:
            e = tmp
        del tmp
    flags = torch.empty(n, dtype=torch.int64, device=dev)
    _lib.call("dr_hi_flags", ptr(e), c_u32(words), c_u64(n), ptr(flags), stream_of(e))
    seg, nseg, starts = _ids_from_flags(flags)
    del flags
    keys = e[:, 1].index_select(0, starts).add_(mn)
    sp = [(op, None if w is None else StridedCol(e, _PAYLOAD_WORDS[w], words), dtype)
          for (op, _, dtype), w in zip(specs, where)]
    return keys, seg_reduce_multi(None, seg, nseg, sp)


_lib.register_signatures({"dr_hash_aggregate": (c_i32, [vp, c_u64, c_i32, vp, vp, vp, vp, c_u64, vp, vp])})

HASH_AGG_MAX_KEYS = 1 << 15


def estimate_distinct(col: torch.Tensor, sample: int = 1 << 16) -> tuple[int, int]:
    """(distinct keys in an evenly strided sample, sample size)."""
    n = col.shape[0]
    if n == 0:
        return 0, 0
    step = max(1, n // sample)
    s_ = col[::step][:sample]
    return int(torch.unique(s_).numel()), int(s_.numel())


def hash_aggregate(key: torch.Tensor, specs: list, capacity: int | None = None):
    """Low-cardinality GroupBy in one streaming pass (csrc/kernels/hashagg.hip).

    ``key``: integer column; ``specs`` as for seg_reduce_multi.  Returns (keys, outs) for the
    distinct keys (unordered), or None when the table overflowed (caller falls back to sorting)."""
    n = key.shape[0]
    dev = key.device
    k64 = key.to(torch.int64).contiguous()
    if capacity is None:
        d, m = estimate_distinct(k64)
        capacity = max(1024, 1 << (max(1, 4 * d) - 1).bit_length())
    gkeys = torch.full((capacity,), -2**63, dtype=torch.int64, device=dev)
    ops, vals, outs, keep = [], [], [], []
    for op, v, dtype in specs:
        f = 0 if dtype in (torch.int64, torch.int32, torch.int16, torch.int8, torch.uint8, torch.bool) else 1
        if op == "count":
            f = 0
        tdt = torch.int64 if f == 0 else torch.float64
        init = {"sum": 0, "count": 0,
                "min": torch.iinfo(torch.int64).max if f == 0 else float("inf"),
                "max": torch.iinfo(torch.int64).min if f == 0 else float("-inf")}[op]
        out = torch.full((capacity + 1,), init, dtype=tdt, device=dev)
        vv = None if op == "count" else v.to(tdt).contiguous()
        keep.append(vv)
        ops.append(_MOPS[(op, f)])
        vals.append(vv.data_ptr() if vv is not None else 0)
        outs.append(out)
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    m = len(specs)
    _lib.call("dr_hash_aggregate", ptr(k64), c_u64(n), m, (ctypes.c_int * m)(*ops), (ctypes.c_void_p * m)(*vals),
              (ctypes.c_void_p * m)(*[o.data_ptr() for o in outs]), ptr(gkeys), c_u64(capacity), ptr(flag),
              stream_of(k64))
    if int(flag.item()):
        return None
    used = torch.nonzero(gkeys != -2**63, as_tuple=False).flatten()
    keys_out = gkeys.index_select(0, used)
    res = [o.index_select(0, used) for o in outs]
    # the INT64_MIN key lives in the extra slot `capacity`
    cnt_special = None
    for (op, _, _), o in zip(specs, outs):
        if op == "count":
            cnt_special = int(o[capacity].item())
            break
    if cnt_special is None:
        cnt_special = int((k64 == -2**63).sum().item())
    if cnt_special:
        keys_out = torch.cat([keys_out, torch.tensor([-2**63], dtype=torch.int64, device=dev)])
        res = [torch.cat([r, o[capacity:capacity + 1]]) for r, o in zip(res, outs)]
    return keys_out.to(key.dtype), res


# ---------------------------------------------------------------------------------------------
# Device image of the host partitioner hash (csrc/kernels/stablehash.hip)
_lib.register_signatures({
    "dr_stable_hash_dest": (c_i32, [ctypes.POINTER(c_i32), ctypes.POINTER(vp), ctypes.POINTER(vp), ctypes.POINTER(vp),
                                    ctypes.POINTER(c_u32), ctypes.POINTER(c_u32), ctypes.POINTER(c_u32), c_i32, c_i32,
                                    c_u64, c_u32, vp, vp, vp, vp]),
})

H_BYTES, H_STR = 20, 21
MAX_HASH_COLS = 8


class HashKey:
    """One field of a key for stable_hash_dest: a typed column, a byte-string field of fixed-width
    rows, or a string field (heap, offsets, lengths)."""
    __slots__ = ("kind", "t", "off", "len", "stride", "boff", "blen")

    def __init__(self, kind, t, off=None, ln=None, stride=0, boff=0, blen=0):
        self.kind, self.t, self.off, self.len = kind, t, off, ln
        self.stride, self.boff, self.blen = stride, boff, blen

    @staticmethod
    def column(c: torch.Tensor) -> "HashKey":
        if c.dtype not in KEY_TYPES or c.dim() != 1:
            raise TypeError(f"hash key column of dtype {c.dtype} / dim {c.dim()}")
        return HashKey(KEY_TYPES[c.dtype], c.contiguous())

    @staticmethod
    def bytes_field(rows: torch.Tensor, off: int, length: int) -> "HashKey":
        assert rows.dtype == torch.uint8 and rows.dim() == 2 and rows.is_contiguous()
        assert 0 <= off and off + length <= rows.shape[1]
        return HashKey(H_BYTES, rows, stride=rows.shape[1], boff=off, blen=length)

    @staticmethod
    def string(heap: torch.Tensor, off: torch.Tensor, ln: torch.Tensor) -> "HashKey":
        if heap.numel() == 0:
            heap = torch.zeros(8, dtype=torch.uint8, device=off.device)
        return HashKey(H_STR, heap, off.to(torch.int64).contiguous(), ln.to(torch.int64).contiguous())


def stable_hash_dest(keys: list, n: int, nparts: int, tuple_form: bool, device,
                     want_hash: bool = False, ports: bool = False):
    """Destination partition of every record under the host partitioner hash
    (runtime/vertex_ops.stable_hash): -> (E128 entries {lo = row, hi = port} or None,
    int64 hashes or None).  ``tuple_form``: the key is a tuple/record of ``keys``.  ``ports``
    (nparts <= 256): one uint8 port per row instead of the 16-byte entries."""
    if not keys or len(keys) > MAX_HASH_COLS or (not tuple_form and len(keys) != 1):
        raise ValueError("stable_hash_dest: 1..8 key fields (exactly 1 unless tuple_form)")
    if n >= (1 << 32):
        raise ValueError("stable_hash_dest: partition of 2^32 rows or more")
    k = len(keys)
    kinds = (c_i32 * k)(*[x.kind for x in keys])
    ptrs = (vp * k)(*[x.t.data_ptr() for x in keys])
    offs = (vp * k)(*[x.off.data_ptr() if x.off is not None else 0 for x in keys])
    lens = (vp * k)(*[x.len.data_ptr() if x.len is not None else 0 for x in keys])
    strides = (c_u32 * k)(*[x.stride for x in keys])
    boffs = (c_u32 * k)(*[x.boff for x in keys])
    blens = (c_u32 * k)(*[x.blen for x in keys])
    if ports and not 0 < nparts <= 256:
        raise ValueError("stable_hash_dest: uint8 ports need 1..256 partitions")
    ent = torch.empty((n, 2), dtype=torch.int64, device=device) if nparts and not ports else None
    pt = torch.empty(n, dtype=torch.uint8, device=device) if ports else None
    hs = torch.empty(n, dtype=torch.int64, device=device) if want_hash else None
    _lib.call("dr_stable_hash_dest", kinds, ptrs, offs, lens, strides, boffs, blens, k, int(bool(tuple_form)),
              c_u64(n), c_u32(nparts), ptr(ent) if ent is not None else None,
              ptr(hs) if hs is not None else None, ptr(pt) if pt is not None else None, stream_of(keys[0].t))
    return (pt if ports else ent), hs


# ---------------------------------------------------------------------------------------------
# Narrow integer keys: compact 8-byte sort whose last pass expands to E128
_lib.register_signatures({
    "dr_build_keys64": (c_i32, [vp, c_i32, c_u64, c_u64, c_u32, vp, vp]),
    "dr_sort_u64_expand": (c_i32, [vp, vp, vp, c_u64, c_i32, c_i32, c_u64, vp, vp]),
})
_INT_BITS = {torch.uint8: 8, torch.int8: 8, torch.bool: 8, torch.int16: 16, torch.uint16: 16, torch.int32: 32,
             torch.uint32: 32, torch.int64: 64, torch.uint64: 64}
_SIGNED = {torch.int8, torch.int16, torch.int32, torch.int64}
INT_KEY_SORT = True


def _norm_int(v: int, dtype) -> int:
    """Order-preserving unsigned image of an integer key (relational.hip norm_key)."""
    b = _INT_BITS[dtype]
    v &= (1 << b) - 1
    return v ^ (1 << (b - 1)) if dtype in _SIGNED else v


def int_key_sort(col: torch.Tensor):
    """Stable sort of one integer key column whose value span is below 2^32, through 8-byte
    entries ((key - min) << 32 | row; half the bytes per radix pass of the 16-byte sort).  Returns
    E128 entries {lo = row, hi = normalised key} (segment_ids / seg_reduce layout, lo_mask 0), or
    None when the column does not qualify."""
    from . import reduce as RD
    from . import sort as S
    n = col.shape[0]
    if not INT_KEY_SORT or col.dtype not in _INT_BITS or col.dim() != 1 or n < 2 or n >= (1 << 32):
        return None
    col = col.contiguous()
    c = col.to(torch.int64) if col.dtype in (torch.bool, torch.uint16, torch.uint32) else col
    mn, mx = RD.reduce_multi(n, [(RD.MIN, c, None), (RD.MAX, c, None)], col.device)
    span = int(mx) - int(mn)
    if span >= (1 << 32):
        return None
    passes = max(1, (span.bit_length() + 7) // 8)
    bias = _norm_int(int(mn), col.dtype)
    dev = col.device
    e = torch.empty(n, dtype=torch.int64, device=dev)
    tmp = torch.empty(n, dtype=torch.int64, device=dev)
    out = torch.empty((n, 2), dtype=torch.int64, device=dev)
    _lib.call("dr_build_keys64", ptr(col), KEY_TYPES[col.dtype], c_u64(n), c_u64(bias), c_u32(0), ptr(e),
              stream_of(col))
    ws = S._workspace(n, dev)
    _lib.call("dr_sort_u64_expand", ptr(e), ptr(tmp), ptr(out), c_u64(n), 32, 32 + 8 * passes, c_u64(bias), ptr(ws),
              stream_of(col))
    return out

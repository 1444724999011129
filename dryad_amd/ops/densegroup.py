"""Dense-key GroupBy aggregation (csrc/kernels/densegroup.hip): two stable partition passes over
bit-packed 16-byte rows by key bits, then one LDS table per run of 2^12 consecutive keys.

Applies to one integer key whose value span needs 13..32 bits (2^12 < span <= 2^32: at most two
partition passes of <= 10 bits) and <= 3 integer value columns whose spans, with the key's, pack
into 128 bits; count / sum / min / max aggregates.  Reference: the partial / full hash GroupBy of
DryadLinqVertex.cs:5342-6417 (ParallelHashGroupBy) -- here the hash table is an LDS table addressed
directly by the low key bits, reached by partitioning on the high ones.

Returns (keys int64, [per-spec int64 column]) in unspecified group order, or None when the shape
does not apply (the caller then takes the radix-aggregation or sort path).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import c_i32, c_i64, c_u32, c_u64, ptr, stream_of, vp

_lib.register_signatures({
    "dr_dg_table_bits": (c_u32, []),
    "dr_dg_max_digit": (c_u32, []),
    "dr_dg_grid": (c_u32, [c_u64, ctypes.POINTER(c_u64)]),
    "dr_dg_count": (c_i32, [vp, vp, c_u64, c_i64, c_u32, c_u32, c_u32, vp, c_u32, c_u64, vp, c_u32, vp]),
    "dr_dg_scatter": (c_i32, [vp, ctypes.POINTER(vp), ctypes.POINTER(c_i64), ctypes.POINTER(c_u32), c_u32, c_i64,
                              c_u32, vp, c_u64, c_u32, c_u32, vp, c_u32, c_u64, vp, vp]),
    "dr_dg_aggregate": (c_i32, [vp, vp, vp, c_u32, c_u32, c_i64, c_u32, ctypes.POINTER(c_u32), ctypes.POINTER(c_u32),
                                ctypes.POINTER(c_u32), ctypes.POINTER(c_i64), vp, vp, vp, ctypes.POINTER(vp), c_i32, vp]),
})

TABLE_BITS = 12
# aggregation workgroups (one per CU by LDS: 1024 = four rounds over the 256 CUs)
AGG_GRID = 1024
MAX_DIGIT = 10                   # the library's dr_dg_max_digit() when it is loaded
_MAXD = None
MIN_ROWS = 1 << 20
_INT = (torch.int64, torch.int32, torch.int16, torch.int8, torch.uint8)
_OP = {"sum": 0, "min": 1, "max": 2}


def plan(kspan_bits: int, vbits: list) -> list | None:
    """Digit widths of the partition passes (low digit first) for a key offset of ``kspan_bits``
    bits, or None when the dense path does not apply."""
    global _MAXD
    if _MAXD is None:
        _MAXD = int(_lib.lib().dr_dg_max_digit()) if torch.cuda.is_available() else MAX_DIGIT
    m = _MAXD
    d = kspan_bits - TABLE_BITS
    if d < 1 or d > 2 * m or kspan_bits + sum(vbits) > 128:
        return None
    if d <= m:
        return [d]
    lo = (d + 1) // 2
    return [lo, d - lo]


def _bits(span: int) -> int:
    return max(1, int(span).bit_length())


def applicable(key: torch.Tensor, specs: list) -> bool:
    return _prepare(key, specs) is not None


def _same_column(a: torch.Tensor, b: torch.Tensor) -> bool:
    """The same column even when the traced lambdas produced distinct tensor objects (e.g.
    Sum / Min / Max of r[1]): one packed field and one column read serve all of them."""
    return a is b or (a.dtype == b.dtype and a.shape == b.shape and a.stride() == b.stride()
                      and a.device == b.device and a.data_ptr() == b.data_ptr())


def _prepare(key: torch.Tensor, specs: list):
    from ..gpu import stats
    n = key.shape[0]
    if key.dim() != 1 or key.dtype not in _INT or n < 2 or n >= (1 << 32):
        return None
    cols, accs, where = [], [], []
    for op, vals, dtype in specs:
        if op == "count":
            where.append(("count", None))
            continue
        if op not in _OP or vals is None or vals.dtype not in _INT or dtype not in _INT:
            return None
        j = next((j for j, c in enumerate(cols) if _same_column(c, vals)), None)
        if j is None:
            if len(cols) == 3:
                return None
            cols.append(vals)
            j = len(cols) - 1
        a = (_OP[op], j)
        if a not in accs:
            if len(accs) == 3:
                return None
            accs.append(a)
        where.append(("acc", accs.index(a)))
    bnds = stats.bounds([key] + cols)
    (kmin, kmax), vb = bnds[0], bnds[1:]
    kbits = _bits(kmax - kmin)
    vbits = [_bits(hi - lo) for lo, hi in vb]
    widths = plan(kbits, vbits)
    if widths is None:
        return None
    # int64 results: a sum's magnitude is bounded by n * max|v|
    for (op, j) in accs:
        lo, hi = vb[j]
        if op == 0 and n * max(abs(lo), abs(hi)) >= (1 << 63):
            return None
    return cols, accs, where, kmin, kbits, [lo for lo, _ in vb], vbits, widths


def _partition(key64, cols64, vmin, vbits, kmin, kbits, src, n, shift, dbits, dev, st, lo_bits=0, need_runs=True):
    """One stable partition pass -> (rows [n, 16 bytes], run sizes int64 on the device).  Run sizes
    (runs = key offset >> TABLE_BITS in the final order) come from the histogram itself on a single
    pass, from the joint (digit, previous digit) count of a second pass (``lo_bits`` = the first
    pass's digit bits)."""
    pb = c_u64(0)
    G = int(_lib.lib().dr_dg_grid(c_u64(n), ctypes.byref(pb)))
    nb = 1 << dbits
    counts = torch.empty(nb * G, dtype=torch.int32, device=dev)
    joint = torch.zeros(nb << lo_bits, dtype=torch.int32, device=dev) if src is not None else None
    _lib.call("dr_dg_count", ptr(key64) if src is None else None, ptr(src), c_u64(n), c_i64(kmin), c_u32(kbits),
              c_u32(shift), c_u32(dbits), ptr(counts), c_u32(G), pb, ptr(joint), c_u32(lo_bits), st)
    c64 = counts.to(torch.int64)
    del counts
    offs = torch.cumsum(c64, 0)
    offs -= c64
    out = torch.empty((n, 2), dtype=torch.int64, device=dev)
    k = len(cols64)
    cp = (vp * 3)(*([c.data_ptr() for c in cols64] + [0] * (3 - k)))
    vm = (c_i64 * 3)(*(list(vmin) + [0] * (3 - k)))
    vbt = (c_u32 * 3)(*(list(vbits) + [0] * (3 - k)))
    _lib.call("dr_dg_scatter", ptr(key64), cp, vm, vbt, c_u32(k), c_i64(kmin), c_u32(kbits), ptr(src), c_u64(n),
              c_u32(shift), c_u32(dbits), ptr(offs), c_u32(G), pb, ptr(out), st)
    if joint is not None:
        runs = joint.to(torch.int64)
    else:
        runs = c64.view(nb, G).sum(1) if need_runs else None
    return out, runs


def dense_aggregate(key: torch.Tensor, specs: list, force: bool = False, agg_grid: int = AGG_GRID):
    """GroupBy on one integer key column through the dense-key path; see the module docstring.
    ``agg_grid``: workgroups of the aggregation kernel (an argument, for A/B tools only)."""
    n = key.shape[0]
    if not key.is_cuda or (not force and n < MIN_ROWS):
        return None
    prep = _prepare(key, specs)
    if prep is None:
        return None
    cols, accs, where, kmin, kbits, vmin, vbits, widths = prep
    dev = key.device
    st = stream_of(key)
    key64 = key if key.dtype == torch.int64 else key.to(torch.int64)
    key64 = key64.contiguous()
    cols64 = [(c if c.dtype == torch.int64 else c.to(torch.int64)).contiguous() for c in cols]
    # pass 1 packs the columns (low digit), pass 2 (if any) re-partitions the rows (high digit)
    # (LSD order: the rows end up sorted by run id = key offset >> TABLE_BITS)
    rows, runs = _partition(key64, cols64, vmin, vbits, kmin, kbits, None, n, TABLE_BITS, widths[0], dev, st,
                            need_runs=len(widths) == 1)
    if len(widths) == 2:
        nxt, runs = _partition(key64, cols64, vmin, vbits, kmin, kbits, rows, n, TABLE_BITS + widths[0], widths[1],
                               dev, st, lo_bits=widths[0])
        del rows
        rows = nxt
    # run r's rows: rstart[r] .. rstart[r + 1]; workgroup g folds the runs starting in its share
    rstart = torch.zeros(runs.shape[0] + 1, dtype=torch.int64, device=dev)
    torch.cumsum(runs, 0, out=rstart[1:])
    G = max(1, min(int(agg_grid), n // 4096))
    targets = torch.arange(G + 1, dtype=torch.int64, device=dev) * ((n + G - 1) // G)
    wrun = torch.searchsorted(rstart[:-1].contiguous(), targets)
    # field offsets of the accumulated columns inside the packed row
    foff, o = [], kbits
    for b in vbits:
        foff.append(o)
        o += b
    head = torch.zeros(1, dtype=torch.int64, device=dev)
    okey = torch.empty(n, dtype=torch.int64, device=dev)
    ocnt = torch.empty(n, dtype=torch.int64, device=dev)
    oacc = [torch.empty(n, dtype=torch.int64, device=dev) for _ in accs]
    na = len(accs)
    ops = (c_u32 * 3)(*([a[0] for a in accs] + [0] * (3 - na)))
    offs = (c_u32 * 3)(*([foff[a[1]] for a in accs] + [0] * (3 - na)))
    bts = (c_u32 * 3)(*([vbits[a[1]] for a in accs] + [0] * (3 - na)))
    vms = (c_i64 * 3)(*([vmin[a[1]] for a in accs] + [0] * (3 - na)))
    optr = (vp * 3)(*([t.data_ptr() for t in oacc] + [0] * (3 - na)))
    # a Sum of a field of <= 32 bits carries the count in its slot's top 16 bits (needs runs of
    # fewer than 2^16 rows, so no slot's count can reach that field)
    ps = next((j for j, a in enumerate(accs) if a[0] == 0 and vbits[a[1]] <= 32), None)
    pack = 0 if ps is None or int(runs.max().item()) >= (1 << 16) else ps + 1
    _lib.call("dr_dg_aggregate", ptr(rows), ptr(rstart), ptr(wrun), c_u32(G), c_u32(kbits), c_i64(kmin), c_u32(na),
              ops, offs, bts, vms, ptr(head), ptr(okey), ptr(ocnt), optr, pack, st)
    del rows
    g = int(head.item())
    keys, cnt = okey[:g], ocnt[:g]
    outs = []
    for kind, i in where:
        outs.append(cnt if kind == "count" else oacc[i][:g])
    if key.dtype != torch.int64:
        keys = keys.to(key.dtype)
    return keys, outs


_lib.register_signatures({
    "dr_dense_state_update": (c_i32, [vp, c_u32, c_u64, c_i64, c_u64, vp, ctypes.POINTER(vp), ctypes.POINTER(vp),
                                      ctypes.POINTER(c_u32), ctypes.POINTER(c_u32), ctypes.POINTER(c_u32), c_u32, c_u64,
                                      vp, vp]),
})
_DS_KEY = {torch.int64: 0, torch.int32: 2, torch.int8: 3, torch.int16: 5}
_DS_VAL = {torch.int64: 0, torch.float64: 1, torch.int32: 2, torch.int8: 3, torch.float32: 4, torch.int16: 5}
_DS_OP = {"count": 0, "sum": 1, "min": 2, "max": 3}


def dense_state_ok(specs: list, key: torch.Tensor, stride: int = 1) -> bool:
    """Can dense_state_update fold these accumulators?  specs: [(state, op, value or None)]: int64
    states with any op, float64 states with sums, values of the listed dtypes; every state a
    column of ``stride``-element rows."""
    if not key.is_cuda or key.dtype not in _DS_KEY or len(specs) > 8:
        return False
    if any(st.dim() != 1 or st.stride(0) != stride for st, _, _ in specs):
        return False
    for st, op, v in specs:
        if st.dtype == torch.int64:
            pass
        elif not (st.dtype == torch.float64 and op == "sum"):
            return False
        if op != "count" and (v is None or v.dtype not in _DS_VAL or not v.is_contiguous()):
            return False
    return key.is_contiguous()


def dense_state_update(key: torch.Tensor, lo: int, seen, specs: list, rng: int | None = None,
                       stride: int = 1) -> None:
    """One pass over the rows: seen[key - lo] = 1 (``seen`` may be None) and every accumulator's
    atomic into its slot (runtime/stream_agg.DenseState); the states are columns of
    ``stride``-element rows (an [R, stride] matrix: a key's slots in one sector).  Raises if a key
    falls outside the state's ``rng`` keys."""
    _lib.require_gpu_tensor(key, "dense_state_update")
    n, k = key.shape[0], len(specs)
    states = (vp * k)(*[st.data_ptr() for st, _, _ in specs])
    vals = (vp * k)(*[(v.data_ptr() if v is not None else None) for _, _, v in specs])
    ops = (c_u32 * k)(*[_DS_OP[op] for _, op, _ in specs])
    sdt = (c_u32 * k)(*[0 if st.dtype == torch.int64 else 1 for st, _, _ in specs])
    vdt = (c_u32 * k)(*[_DS_VAL[v.dtype] if v is not None else 0 for _, _, v in specs])
    bad = torch.zeros(1, dtype=torch.int32, device=key.device)
    rng = seen.numel() if rng is None else rng
    _lib.call("dr_dense_state_update", ptr(key), c_u32(_DS_KEY[key.dtype]), c_u64(n), c_i64(lo), c_u64(rng),
              ptr(seen) if seen is not None else None, states, vals, ops, sdt, vdt, c_u32(k), c_u64(stride), ptr(bad),
              stream_of(key))
    if int(bad.item()):
        raise RuntimeError("dense_state_update: a key outside the state's range")

"""GPU implementations of the vertex operator library over HBM-resident ``DeviceTable`` partitions.

Each function mirrors an op of ``runtime/vertex_ops.py`` (the object path) with the same
signature ``fn(op, inputs, vctx)``; inputs are DeviceTables, the result a DeviceTable or a
``Ported`` table for multi-port (partitioning) outputs.  An op raises ``NotTraceable`` when it
cannot run on the device (opaque lambda, custom comparer, string data, ...); the executor then runs
the object implementation for that op only.

Hot paths are HIP kernels: key normalisation (dr_build_keys / dr_extract_keys), LSD radix sort
(dr_sort_u128), hashing and partition passes (dr_hash_dest / dr_partition_pass_u128), range
destinations (dr_range_dest_u128), segmented reductions (dr_seg_reduce), merge-join expansion
(dr_join_ranges / dr_join_emit), row gathers (dr_gather_rows) and the synthetic TeraSort store.
Elementwise projections/predicates are traced user lambdas executed as PyTorch-ROCm tensor ops.
"""
from __future__ import annotations

import torch

from ..compiler.decomposition import Sym, substitute
from ..ops import recordsort as RS
from ..ops import relational as R
from ..ops import sort as S
from . import trace as TR
from .table import DeviceTable, PartialMeta, Ported, Shape, from_objects
from .trace import NotTraceable

E_SHAPE = Shape("tuple", ["lo", "hi"])


def _one(inputs) -> DeviceTable:
    ts = [t for t in inputs if t is not None]
    if len(ts) == 1:
        return ts[0]
    return DeviceTable.concat(ts)


def _check(t):
    if not isinstance(t, DeviceTable):
        raise NotTraceable("host partition")
    return t


# ---------------------------------------------------------------------------------------------
# key handling
def key_entries(table: DeviceTable, key_fn, comparer=None, descending=False):
    """-> (entries [n,2], begin_bit, lo_mask).  Keys compare like the object path's default order."""
    if table.heap is not None:
        raise NotTraceable("string keys")
    if comparer is not None:
        raise NotTraceable("custom comparer")
    if table.n == 0:
        return torch.empty((0, 2), dtype=torch.int64, device=table.device), 64, 0
    res = TR.call(key_fn, table)
    kind, spec = TR.key_columns(res, table)
    if kind == "bytes":
        if spec.length > 12:
            raise NotTraceable("byte key longer than 12 bytes")
        e = S.extract_keys(table.rows, spec.off, spec.length, 0)
        b0, _, lo_mask = RS.key_bits(spec.length)
        if descending:
            e[:, 1].bitwise_not_()
            if lo_mask:
                e[:, 0].bitwise_xor_(torch.tensor(RS._as_i64(lo_mask), dtype=torch.int64, device=e.device))
        return e, b0, lo_mask
    cols = spec
    for c in cols:
        if c.dtype not in R.KEY_TYPES:
            raise NotTraceable(f"key dtype {c.dtype}")
    if R.key_bit_count(cols) > 96:
        raise NotTraceable("composite key wider than 96 bits")
    e, b0, lo_mask = R.build_keys(cols, [descending] * len(cols))
    return e, b0, lo_mask


def eq_key_entries(table: DeviceTable, key_fn, comparer=None):
    """Entries for equality-only consumers (HashPartition, Join): like key_entries, but string
    fields are keyed by their Rabin-64 fingerprints.  -> (entries, begin_bit, lo_mask, skeys)."""
    if table.heap is not None:
        raise NotTraceable("text records")
    if comparer is not None:
        raise NotTraceable("custom comparer")
    if table.n == 0:
        return torch.empty((0, 2), dtype=torch.int64, device=table.device), 64, 0, []
    res = TR.call(key_fn, table)
    try:
        kind, spec = TR.key_columns(res, table)
    except NotTraceable:
        kind = "str"
    if kind != "str":
        e, b0, lo_mask = key_entries(table, key_fn, comparer)
        return e, b0, lo_mask, []
    cols, skeys = TR.eq_key_columns(res, table)
    for c in cols:
        if c.dtype not in R.KEY_TYPES:
            raise NotTraceable(f"key dtype {c.dtype}")
    if R.key_bit_count(cols) > 96:
        raise NotTraceable("composite key wider than 96 bits")
    e, b0, lo_mask = R.build_keys(cols)
    return e, b0, lo_mask, skeys


def _perm(entries: torch.Tensor) -> torch.Tensor:
    return (entries[:, 0] & 0xFFFFFFFF).contiguous()


def sort_perm(table, key_fn, comparer=None, descending=False):
    e, b0, lo_mask = key_entries(table, key_fn, comparer, descending)
    srt = S.sort_entries_hybrid(e, b0)
    return srt, _perm(srt), lo_mask


# ---------------------------------------------------------------------------------------------
# sources / trivial ops
def op_enumerable(op, inputs, v):
    recs = op["chunks"][v.partition]
    t = from_objects(recs, op.get("dtype"), v.device)
    if t is None:
        raise NotTraceable("non-columnar record type")
    return t


def op_read(op, inputs, v):
    from ..io.providers import parse_uri, provider_for
    uri = op["uri"]
    scheme, path, q = parse_uri(uri)
    if scheme == "gen":
        kind = path.strip("/")
        from ..io.providers import GenProvider
        lo, hi = GenProvider().bounds(uri, v.partition)
        if kind == "terasort":
            from ..ops import terasort as TSK
            rows = v.alloc_rows(hi - lo, 100)
            t = DeviceTable(hi - lo, Shape("rows", key_off=0, key_len=10), rows=rows)
            bs = _pooled_set(t, v)
            if bs is not None:
                # producer-side key extraction: a following OrderBy(key bytes 0..9) starts sorting
                rng = torch.tensor([-1, 0], dtype=torch.int64, device=rows.device)
                TSK.generate_with_keys(rows, lo, int(q.get("seed", 0)), bs.bufs.ent_a, rng)
                bs.keys_ready = (rows.data_ptr(), hi - lo, 0, 10, rng)
            else:
                TSK.generate(rows, lo, int(q.get("seed", 0)))
            return t
        if kind == "points":
            from ..ops import kmeans as KM
            x = v.alloc_tensor((hi - lo, KM.DIM), torch.float32)
            KM.generate(x, lo, int(q.get("blobs", 64)), int(q.get("seed", 0)))
            from .. import types as T
            return DeviceTable.from_columns({"x": x}, Shape("vector", ["x"], T.Vector(T.Float32, KM.DIM)))
        if kind == "records64":
            from ..ops import relational as R
            from ..models.records_cpu import FIELDS
            ncols = int(q.get("cols", 8))
            cols = [v.alloc_tensor((hi - lo,), torch.int64) for _ in range(ncols)]
            from ..models.records_cpu import dim_multiplier
            nk = int(q.get("keys", 1 << 20))
            R.gen_records64(cols, lo, nk, int(q.get("seed", 0)), dim_multiplier(nk) if q.get("mode") == "dim" else 0)
            names = FIELDS[:ncols]
            return DeviceTable.from_columns(dict(zip(names, cols)), Shape("tuple", names))
        if kind == "range":
            start = int(q.get("start", 0))
            a = torch.arange(start + lo, start + hi, dtype=torch.int32 if start + hi < 2**31 else torch.int64,
                             device=v.device)
            return DeviceTable.from_columns({"v": a}, Shape("scalar", ["v"]))
    if scheme == "hbm":
        return provider_for(uri).get(uri)["local"][v.partition]
    if scheme == "text":
        # raw bytes -> HBM heap -> line (offset, length) pairs on the device
        from ..ops import text as TX
        from .table import text_table
        from .. import types as T
        data = provider_for(uri).read_partition_bytes(uri, v.partition)
        heap = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(v.device) if data else \
            torch.zeros(0, dtype=torch.uint8, device=v.device)
        off, ln = TX.lines(heap)
        t = text_table(heap, off, ln, T.LineRecord)
        t.whole_heap = True           # every line of the heap, in order (tokenise the heap directly)
        return t
    prov = provider_for(uri)
    if scheme in ("partfile", "file") and v.device.type == "cuda":
        # binary part of fixed-width records: bytes -> HBM -> columns with the device codec
        from ..ops import codec as CD
        sch = prov.schema(uri) or {}
        dt = op.get("dtype") or sch.get("dtype")
        if sch.get("format", "binary") == "binary" and dt is not None and CD.layout(dt) is not None:
            data = prov.read_partition_bytes(uri, v.partition)
            buf = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(v.device) if data else \
                torch.zeros(0, dtype=torch.uint8, device=v.device)
            t = CD.decode(buf, dt)
            if t is not None:
                return t
    recs = prov.read_partition(uri, v.partition, op.get("dtype"))
    t = from_objects(recs, op.get("dtype"), v.device)
    if t is None:
        raise NotTraceable("non-columnar store records")
    return t


def op_identity(op, inputs, v):
    return _one(inputs)


def op_concat(op, inputs, v):
    return _one(inputs)


def op_output(op, inputs, v):
    return _one(inputs)


def op_where(op, inputs, v):
    t = _check(_one(inputs))
    if t.n == 0:
        return t
    return t.mask(TR.to_mask(TR.call(op["fn"], t), t))


def op_select(op, inputs, v):
    t = _check(_one(inputs))
    if t.n == 0:
        raise NotTraceable("empty partition: output type unknown")
    return TR.to_table(TR.call(op["fn"], t), t)


def _offset(inputs, v):
    offs = inputs[1]
    if isinstance(offs, DeviceTable):
        vals = offs.cols[offs.shape.fields[0]].tolist()
    else:
        vals = list(offs)
    return vals[v.partition] if v.partition < len(vals) else 0


def op_where_idx(op, inputs, v):
    t = _check(inputs[0])
    if t.n == 0:
        return t
    return t.mask(TR.to_mask(TR.call(op["fn"], t, _offset(inputs, v)), t))


def op_select_idx(op, inputs, v):
    t = _check(inputs[0])
    if t.n == 0:
        raise NotTraceable("empty partition")
    return TR.to_table(TR.call(op["fn"], t, _offset(inputs, v)), t)


def op_take(op, inputs, v):
    t = _check(_one(inputs))
    return t.slice(0, min(t.n, max(0, op["count"])))


def op_skip(op, inputs, v):
    t = _check(_one(inputs))
    return t.slice(min(t.n, max(0, op["count"])), t.n)


def op_reverse(op, inputs, v):
    t = _check(_one(inputs))
    return t.take(torch.arange(t.n - 1, -1, -1, device=t.device))


def _scalar_table(vals, dtype, device):
    return DeviceTable.from_columns({"v": torch.tensor(vals, dtype=dtype, device=device)}, Shape("scalar", ["v"]))


def op_count(op, inputs, v):
    t = _check(_one(inputs))
    return _scalar_table([t.n], torch.int64, v.device)


def op_offsets(op, inputs, v):
    t = _check(_one(inputs))
    c = t.cols[t.shape.fields[0]].to(torch.int64)
    return DeviceTable.from_columns({"v": torch.cumsum(c, 0) - c}, Shape("scalar", ["v"]))


# ---------------------------------------------------------------------------------------------
# sorting / partitioning
def _pooled_set(t: DeviceTable, v):
    """The executor's pooled buffer set whose rows_in holds this row table (or None)."""
    r = getattr(v, "runner", None)
    if r is None or t.rows is None:
        return None
    bs = r.row_sets.get((v.stage.id, v.partition))
    if bs is not None and t.rows.data_ptr() == bs.bufs.rows_in.data_ptr():
        return bs
    return None


def op_sort(op, inputs, v):
    t = _check(_one(inputs))
    if t.n <= 1:
        return t
    bs = _pooled_set(t, v)
    if bs is not None and op.get("comparer") is None:
        # in-place key-pointer sort of pooled rows: rows_in -> rows_out, entries in the pool
        kind, spec = TR.key_columns(TR.call(op["key"], t), t)
        if kind == "bytes" and spec.length <= 12:
            bounds = bs.take_keys(t.rows, spec.off, spec.length)
            out = RS.local_sort_rows(t.rows, bs.bufs.rows_out, bs.bufs.ent_a, bs.bufs.ent_b, spec.off, spec.length,
                                     descending=op.get("descending", False), hi_bounds=bounds,
                                     keys_ready=bounds is not None)
            return DeviceTable(out.shape[0], t.shape, rows=out)
    _, perm, _ = sort_perm(t, op["key"], op.get("comparer"), op.get("descending", False))
    return t.take(perm)


def op_hash_partition(op, inputs, v):
    t = _check(_one(inputs))
    n = op["count"]
    if op.get("comparer") is not None:
        raise NotTraceable("custom comparer")
    if t.n == 0:
        return Ported(t, [0] * (n + 1))
    e, _, lo_mask, _ = eq_key_entries(t, op["key"])
    R.hash_dest(e, lo_mask, n)
    part, starts = S.partition_pass(e, 64)
    st = starts[: n + 1].tolist()
    return Ported(t.take(_perm(part)), st)


def op_sample(op, inputs, v):
    t = _check(_one(inputs))
    e, b0, lo_mask = key_entries(t, op["key"], op.get("comparer"), False)
    n = t.n
    rate = op.get("rate", 0.001)
    m = n if n * rate < 10 else max(1, int(n * rate))
    stride = max(1, n // max(m, 1))
    samp = e[::stride][:m].clone() if n else e
    samp[:, 0] &= RS._as_i64(lo_mask)
    return DeviceTable.from_columns({"lo": samp[:, 0].contiguous(), "hi": samp[:, 1].contiguous()}, E_SHAPE)


def op_separators(op, inputs, v):
    t = _check(_one(inputs))
    n = op["count"]
    if t.n == 0:
        return DeviceTable.from_columns({"lo": torch.empty(0, dtype=torch.int64, device=v.device),
                                         "hi": torch.empty(0, dtype=torch.int64, device=v.device)}, E_SHAPE)
    e = torch.stack([t.cols["lo"], t.cols["hi"]], 1).contiguous()
    srt = S.sort_entries(e, 0, 128)
    pos = torch.tensor([(j * t.n) // n for j in range(1, n)], dtype=torch.int64, device=e.device)
    s = srt.index_select(0, pos)
    return DeviceTable.from_columns({"lo": s[:, 0].contiguous(), "hi": s[:, 1].contiguous()}, E_SHAPE)


def op_range_partition(op, inputs, v):
    t = _check(inputs[0])
    n = op["count"]
    if op.get("separators") is not None:
        raise NotTraceable("explicit separators are host values")
    seps_t = inputs[1] if len(inputs) > 1 else None
    if t.n == 0:
        return Ported(t, [0] * (n + 1))
    e, _, lo_mask = key_entries(t, op["key"], op.get("comparer"), False)
    if seps_t is None or seps_t.n == 0:
        return Ported(t, [0] + [t.n] * n)
    seps = torch.stack([seps_t.cols["lo"], seps_t.cols["hi"]], 1).contiguous()
    S.range_dest(e, seps, lo_mask, descending=op.get("descending", False))
    part, starts = S.partition_pass(e, 64)
    return Ported(t.take(_perm(part)), starts[: n + 1].tolist())


# ---------------------------------------------------------------------------------------------
# GroupBy with decomposable aggregates (sort-based: radix sort -> segments -> segmented reduce)
_GPU_AGGS = {"count", "sum", "min", "max", "avg", "any", "all"}


def _agg_value(agg, t):
    if agg.kind == "count":
        if agg.pred is None:
            return None
        return TR.to_mask(TR.call(agg.pred, t), t).to(torch.int64)
    if agg.kind in ("any", "all"):
        if agg.pred is None:
            return torch.ones(t.n, dtype=torch.int64, device=t.device)
        return TR.to_mask(TR.call(agg.pred, t), t).to(torch.int64)
    if agg.sel is None:
        if t.shape.kind != "scalar":
            raise NotTraceable("aggregate over non-scalar records")
        return t.cols[t.shape.fields[0]]
    r = TR.call(agg.sel, t)
    if not isinstance(r, TR.Col):
        raise NotTraceable("aggregate selector must produce a scalar field")
    return r.t


def _key_cols(t, key_fn):
    """Group key columns; string fields become Rabin fingerprints (skeys[i] = their StrCol).
    Also returns how the host path represents the key ("single" or "tuple")."""
    res = TR.call(key_fn, t)
    if isinstance(res, TR.RecProxy) and t.shape.kind == "dataclass":
        raise NotTraceable("record-valued group key")
    cols, skeys = TR.eq_key_columns(res, t)
    form = "tuple" if isinstance(res, (tuple, TR.RecProxy)) else "single"
    return cols, skeys, form


def _partial_table(out, strs, d, nkeys, form):
    names = [f for f in out if not f.endswith("#len")]
    meta = PartialMeta(nkeys, tuple(a.kind for a in d.aggs), form)
    tb = DeviceTable.from_columns(out, Shape("partial", names, meta))
    tb.strs = strs
    return tb


def _group_keys(kcols, skeys):
    """Sort by the key columns -> (srt, seg, nseg, rows_at_start).  With string keys, every row is
    checked against its group's representative so a fingerprint collision can never merge two
    different strings (the operator falls back to the host if one ever occurs)."""
    e, b0, lo_mask = R.build_keys(kcols)
    srt = S.sort_entries_hybrid(e, b0)
    seg, nseg, starts = R.segment_ids(srt, lo_mask)
    perm = _perm(srt)
    rows_at_start = perm.index_select(0, starts)
    if any(sk is not None for sk in skeys):
        from ..ops.fingerprint import strings_differ
        rep = rows_at_start.index_select(0, seg)          # representative row, in sorted order
        for sk in skeys:
            if sk is not None:
                trip = (sk.heap, sk.off, sk.len)
                if strings_differ(trip, perm, trip, rep):
                    raise NotTraceable("string key fingerprint collision")
    return srt, seg, nseg, rows_at_start


def _key_outputs(kcols, skeys, rows_at_start):
    """Per-group key columns (string keys keep their heap) -> (cols, strs)."""
    out, strs = {}, {}
    for i, (c, sk) in enumerate(zip(kcols, skeys)):
        if sk is None:
            out[f"k{i}"] = c.index_select(0, rows_at_start)
        else:
            out[f"k{i}"] = sk.off.index_select(0, rows_at_start)
            out[f"k{i}#len"] = sk.len.index_select(0, rows_at_start)
            strs[f"k{i}"] = sk.heap
    return out, strs


def _key_values(tb, nkeys):
    """Key columns of a group table as traced values (StrCol for string keys)."""
    vals = []
    for i in range(nkeys):
        f = f"k{i}"
        vals.append(TR.StrCol(tb.strs[f], tb.cols[f], tb.cols[f + "#len"]) if f in tb.strs else tb.cols[f])
    return vals


def _group_specs(d, t):
    """Aggregate specs (op, column, dtype) + output column names of a decomposed GroupBy."""
    specs, names = [], []
    for j, a in enumerate(d.aggs):
        val = _agg_value(a, t)
        if a.kind == "count":
            specs.append(("count", None, torch.int64) if val is None else ("sum", val, torch.int64))
            names.append(f"a{j}")
        elif a.kind in ("sum", "min", "max"):
            specs.append((a.kind, val, val.dtype))
            names.append(f"a{j}")
        elif a.kind == "avg":
            specs += [("sum", val, torch.float64), ("count", None, torch.int64)]
            names += [f"a{j}", f"c{j}"]
        elif a.kind in ("any", "all"):
            specs.append(("max" if a.kind == "any" else "min", val, torch.int64))
            names.append(f"a{j}")
    return specs, names


def op_group_partial(op, inputs, v):
    t = _check(_one(inputs))
    d = op["decomp"]
    if op.get("comparer") is not None or any(a.kind not in _GPU_AGGS for a in d.aggs):
        raise NotTraceable("aggregate not supported on the device")
    if t.n == 0:
        raise NotTraceable("empty partition")
    kcols, skeys, form = _key_cols(t, op["key"])
    specs, names = _group_specs(d, t)
    # low-cardinality integer keys: one streaming pass into LDS hash tables (no sort)
    if len(kcols) == 1 and skeys[0] is None and not kcols[0].is_floating_point() and t.n >= (1 << 16):
        nd, m = R.estimate_distinct(kcols[0])
        if nd <= R.HASH_AGG_MAX_KEYS and nd * 8 < m:
            got = R.hash_aggregate(kcols[0], specs)
            if got is not None:
                keys, res = got
                out = {"k0": keys}
                for nm, r in zip(names, res):
                    out[nm] = r
                return _partial_table(out, {}, d, 1, form)
    srt, seg, nseg, rows_at_start = _group_keys(kcols, skeys)
    out, strs = _key_outputs(kcols, skeys, rows_at_start)
    # every aggregate in one fused segmented-reduce pass
    for nm, res in zip(names, R.seg_reduce_multi(srt, seg, nseg, specs)):
        out[nm] = res
    return _partial_table(out, strs, d, len(kcols), form)


def op_group_final(op, inputs, v):
    t = _check(_one(inputs))
    d = op["decomp"]
    if t.n == 0:
        raise NotTraceable("empty partition")
    if t.shape.kind != "partial":
        raise NotTraceable("group_final input is not a device partial table")
    nkeys = t.shape.pytype.nkeys
    kcols, skeys = TR.eq_key_columns(tuple(TR.Col(v) if isinstance(v, torch.Tensor) else v
                                           for v in _key_values(t, nkeys)), t)
    srt, seg, nseg, rows_at_start = _group_keys(kcols, skeys)
    kout, kstrs = _key_outputs(kcols, skeys, rows_at_start)
    keys = _key_values(DeviceTable(nseg, Shape("tuple", list(kout)), kout, strs=kstrs), nkeys)
    specs = []
    for j, a in enumerate(d.aggs):
        col = t.cols[f"a{j}"]
        if a.kind in ("count", "sum"):
            specs.append(("sum", col, col.dtype))
        elif a.kind in ("min", "max"):
            specs.append((a.kind, col, col.dtype))
        elif a.kind == "avg":
            specs += [("sum", col, torch.float64), ("sum", t.cols[f"c{j}"], torch.int64)]
        elif a.kind in ("any", "all"):
            specs.append(("max" if a.kind == "any" else "min", col, torch.int64))
    res = iter(R.seg_reduce_multi(srt, seg, nseg, specs))
    vals = []
    for j, a in enumerate(d.aggs):
        col = t.cols[f"a{j}"]
        r = next(res)
        if a.kind in ("count", "sum", "min", "max"):
            vals.append(r if col.dtype in (torch.int64, torch.float64) else r.to(col.dtype))
        elif a.kind == "avg":
            vals.append(r / next(res).to(torch.float64))
        else:
            vals.append(r.to(torch.bool))
    return _group_result(d, keys, vals, nseg, t.shape.pytype.key_form)


def _group_result(d, keys, vals, nseg, form="single"):
    """Substitute the per-group key/aggregate columns into the result-selector template."""
    nkeys = len(keys)
    kv = [k if isinstance(k, TR.StrCol) else TR.Col(k) for k in keys]
    key = kv[0] if nkeys == 1 and form == "single" else tuple(kv)
    env = {"key": key, "aggs": [TR.Col(x) for x in vals]}
    try:
        res = substitute(d.template, env)
    except NotTraceable:
        raise
    except Exception as ex:  # noqa: BLE001
        raise NotTraceable(f"result template: {ex}")
    k0 = keys[0].off if isinstance(keys[0], TR.StrCol) else keys[0]
    proto = DeviceTable(nseg, Shape("scalar", ["v"]), {"v": k0})
    return TR.to_table(res, proto)


def op_group_by(op, inputs, v):
    """GroupBy over an already key-partitioned input (e.g. one partition): with a decomposable
    result selector the partial aggregation pass is already the whole answer."""
    d = op.get("decomp")
    if d is None or op.get("elem") is not None:
        raise NotTraceable("non-decomposable GroupBy")
    tb = op_group_partial(dict(op, decomp=d), inputs, v)
    nkeys = tb.shape.pytype.nkeys
    keys = _key_values(tb, nkeys)
    vals = []
    for j, a in enumerate(d.aggs):
        col = tb.cols[f"a{j}"]
        if a.kind == "avg":
            vals.append(col / tb.cols[f"c{j}"].to(torch.float64))
        elif a.kind in ("any", "all"):
            vals.append(col.to(torch.bool))
        else:
            vals.append(col)
    return _group_result(d, keys, vals, tb.n, tb.shape.pytype.key_form)


# ---------------------------------------------------------------------------------------------
def op_distinct(op, inputs, v):
    t = _check(_one(inputs))
    if t.heap is not None or t.strs:
        raise NotTraceable("string records")
    if op.get("comparer") is not None:
        raise NotTraceable("custom comparer")
    if t.n <= 1:
        return t
    if t.rows is not None:
        if t.rows.shape[1] > 12:
            raise NotTraceable("wide rows")
        e, b0, lo_mask = key_entries(t, lambda r: r[0:t.rows.shape[1]])
    else:
        cols = [t.cols[f] for f in t.shape.fields]
        if R.key_bit_count(cols) > 96:
            raise NotTraceable("record wider than 96 bits")
        e, b0, lo_mask = R.build_keys(cols)
    srt = S.sort_entries_hybrid(e, b0)
    _, _, starts = R.segment_ids(srt, lo_mask)
    return t.take(_perm(srt).index_select(0, starts))


def _record_entries(t):
    if t.strs:
        raise NotTraceable("records with string fields")
    if t.rows is not None:
        if t.rows.shape[1] > 12:
            raise NotTraceable("wide rows")
        return key_entries(t, lambda r: r[0:t.rows.shape[1]])
    cols = [t.cols[f] for f in t.shape.fields]
    if R.key_bit_count(cols) > 96:
        raise NotTraceable("record wider than 96 bits")
    e, b0, lo_mask = R.build_keys(cols)
    return e, b0, lo_mask


def _set_op(kind, op, inputs):
    """Union / Intersect / Except (K10): sort the concatenation, segment equal records and keep
    one representative per segment according to which sides the segment contains."""
    if op.get("comparer") is not None:
        raise NotTraceable("custom comparer")
    a, b = _check(inputs[0]), _check(inputs[1])
    if a.heap is not None or b.heap is not None:
        raise NotTraceable("string records")
    if a.shape.kind != b.shape.kind or a.shape.fields != b.shape.fields or a.row_bytes() != b.row_bytes():
        raise NotTraceable("operands have different layouts")
    both = DeviceTable.concat([a, b])
    if both.n == 0:
        return both
    e, b0, lo_mask = _record_entries(both)
    srt = S.sort_entries_hybrid(e, b0)
    seg, nseg, starts = R.segment_ids(srt, lo_mask)
    first = _perm(srt).index_select(0, starts)
    if kind == "union":
        return both.take(first)
    side = (torch.arange(both.n, device=both.device) >= a.n).to(torch.int64)   # 0 = left, 1 = right
    lo_side, hi_side = R.seg_reduce_multi(srt, seg, nseg, [("min", side, torch.int64), ("max", side, torch.int64)])
    keep = (lo_side == 0) & (hi_side == 1) if kind == "intersect" else (hi_side == 0)
    return both.take(first[keep])


def op_union(op, inputs, v):
    return _set_op("union", op, inputs)


def op_intersect(op, inputs, v):
    return _set_op("intersect", op, inputs)


def op_except(op, inputs, v):
    return _set_op("except", op, inputs)


def _while_cut(op, t):
    m = TR.to_mask(TR.call(op["fn"], t, 0 if op.get("indexed") else None), t)
    bad = torch.nonzero(~m, as_tuple=False)
    return int(bad[0].item()) if bad.numel() else t.n


def op_take_while(op, inputs, v):
    t = _check(_one(inputs))
    if t.n == 0:
        return t
    return t.slice(0, _while_cut(op, t))


def op_skip_while(op, inputs, v):
    t = _check(_one(inputs))
    if t.n == 0:
        return t
    return t.slice(_while_cut(op, t), t.n)


def op_hash_join(op, inputs, v):
    outer, inner = _check(inputs[0]), _check(inputs[1])
    if op.get("comparer") is not None:
        raise NotTraceable("custom comparer")
    if outer.n == 0 or inner.n == 0:
        raise NotTraceable("empty join side: output type unknown")
    eo, b0, lm, so_keys = eq_key_entries(outer, op["outer_key"])
    ei, b1, lm2, si_keys = eq_key_entries(inner, op["inner_key"])
    if (b0, lm) != (b1, lm2) or [k is None for k in so_keys] != [k is None for k in si_keys]:
        raise NotTraceable("join keys of different types")
    so = S.sort_entries_hybrid(eo, b0)
    si = S.sort_entries_hybrid(ei, b0)
    oo, ii, _ = R.merge_join_pairs(so, si, lm)
    if oo.shape[0] == 0:
        raise NotTraceable("empty join result")
    if so_keys:
        # string keys matched by fingerprint: every emitted pair must hold equal strings
        from ..ops.fingerprint import strings_differ
        for a, b in zip(so_keys, si_keys):
            if a is not None and strings_differ((a.heap, a.off, a.len), oo, (b.heap, b.off, b.len), ii):
                raise NotTraceable("string key fingerprint collision")
    a, b = outer.take(oo), inner.take(ii)
    res = op["result"](TR.proxy(a), TR.proxy(b))
    return TR.to_table(res, a)


op_merge_join = op_hash_join


# ---------------------------------------------------------------------------------------------
# aggregates: partial per partition (device reductions) -> final on one vertex
def op_agg_partial(op, inputs, v):
    t = _check(_one(inputs))
    s = op["spec"]
    k = s["kind"]
    if s.get("comparer") is not None:
        raise NotTraceable("comparer")
    if k == "Count":
        if s.get("predicate") is None:
            return _scalar_table([t.n], torch.int64, v.device)
        if t.n == 0:
            return _scalar_table([0], torch.int64, v.device)
        return _scalar_table([int(TR.to_mask(TR.call(s["predicate"], t), t).sum().item())], torch.int64, v.device)
    raise NotTraceable(f"aggregate {k} on host")


def op_agg_final(op, inputs, v):
    t = _check(_one(inputs))
    if op["spec"]["kind"] == "Count":
        return _scalar_table([int(t.cols[t.shape.fields[0]].sum().item())], torch.int64, v.device)
    raise NotTraceable("aggregate on host")


def op_apply(op, inputs, v):
    """Apply / ApplyPerPartition: ``@device_function`` bodies run on the HBM tables; any other
    Python body runs on the host records (NotTraceable -> host op)."""
    from ..attributes import is_device_function
    f = op["fn"]
    if not is_device_function(f):
        raise NotTraceable("Apply body is not a @device_function")
    from .. import device_udf
    res = device_udf.call(f, [x if x is not None else [] for x in inputs], op.get("in_dtypes") or [],
                          bool(op.get("multi")), v.device)
    if isinstance(res, DeviceTable):
        return res
    res = list(res)
    out = from_objects(res, None, v.device) if res else None
    return out if out is not None else res      # non-columnar results travel as host records


OPS = {k[3:]: fn for k, fn in list(globals().items()) if k.startswith("op_")}

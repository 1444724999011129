"""GPU implementations of the vertex operator library over HBM-resident ``DeviceTable`` partitions.

Each function mirrors an op of ``runtime/vertex_ops.py`` (the object path) with the same
signature ``fn(op, inputs, vctx)``; inputs are DeviceTables, the result a DeviceTable or a
``Ported`` table for multi-port (partitioning) outputs.  An op raises ``NotTraceable`` when it
cannot run on the device (opaque lambda, custom comparer, string data, ...); the executor then runs
the object implementation for that op only.

Hot paths are HIP kernels: key normalisation (dr_build_keys / dr_extract_keys), LSD radix sort
(dr_sort_u128), hashing and partition passes (dr_hash_dest / dr_partition_pass_u128), range
destinations (dr_range_dest_u128), segmented reductions (dr_seg_reduce), merge-join expansion
(dr_join_ranges / dr_join_emit), the hash join (dr_hj_*), whole-partition aggregates
(dr_reduce_multi), row gathers (dr_gather_rows) and the synthetic TeraSort store.
Elementwise projections/predicates are traced user lambdas executed as PyTorch-ROCm tensor ops.
"""
from __future__ import annotations

import functools

import torch

from ..compiler.decomposition import Sym, substitute
from ..ops import recordsort as RS
from ..ops import relational as R
from ..ops import sort as S
from . import stats
from . import trace as TR
from .table import DeviceTable, PartialMeta, Ported, PortTables, Shape, from_objects
from .trace import NotTraceable
from ..utils.log import get_logger

log = get_logger("gpu.ops")

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
def _row_index_fits(n: int):
    """Sort entries carry a 32-bit row index (low word of ``lo``)."""
    if n >= (1 << 32):
        raise NotTraceable("partition of 2^32 rows or more (32-bit row index in the sort entries)")


def key_entries(table: DeviceTable, key_fn, comparer=None, descending=False):
    """-> (entries [n,2], begin_bit, lo_mask).  Keys compare like the object path's default order."""
    _row_index_fits(table.n)
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


def _wide(cols) -> bool:
    """Key columns that do not fit one 128-bit sort entry (96 key bits + the 32-bit row index)."""
    return len(cols) > 4 or R.key_bit_count(cols) > 96


def _wide_key(cols):
    """Wide key columns -> (int64 Rabin-64 fingerprint of each row's packed key bytes, the packed
    bytes).  -0.0 and 0.0 pack alike (one key, as in Python)."""
    from ..ops.fingerprint import rabin_rows
    parts = []
    for c in cols:
        if c.is_floating_point():
            c = c + 0.0
        parts.append(c.contiguous().view(torch.uint8).reshape(c.shape[0], -1))
    packed = torch.cat(parts, 1).contiguous()
    return rabin_rows(packed), packed


def _rows_differ(pa, ia, pb, ib) -> bool:
    """True if some packed byte row pa[ia[i]] differs from pb[ib[i]] (ia None = identity)."""
    from ..ops.fingerprint import strings_differ

    def trip(p):
        w = p.shape[1]
        off = torch.arange(p.shape[0], dtype=torch.int64, device=p.device) * w
        return p.reshape(-1), off, torch.full_like(off, w)
    return strings_differ(trip(pa), ia, trip(pb), ib)


def eq_key_entries(table: DeviceTable, key_fn, comparer=None):
    """Entries for equality-only consumers (HashPartition, Join): like key_entries, but string
    fields are keyed by their Rabin-64 fingerprints, and keys wider than one 96-bit entry (or byte
    keys longer than 12 bytes) by the fingerprint of their packed bytes.
    -> (entries, begin_bit, lo_mask, skeys, wide): ``wide`` = (packed key bytes, key layout) for a
    fingerprinted wide key (callers that pair rows verify the bytes), else None."""
    _row_index_fits(table.n)
    if table.heap is not None:
        raise NotTraceable("text records")
    if comparer is not None:
        raise NotTraceable("custom comparer")
    if table.n == 0:
        return torch.empty((0, 2), dtype=torch.int64, device=table.device), 64, 0, [], None
    res = TR.call(key_fn, table)
    try:
        kind, spec = TR.key_columns(res, table)
    except NotTraceable:
        kind = "str"
    if kind == "bytes":
        if spec.length <= 12:
            e, b0, lo_mask = key_entries(table, key_fn, comparer)
            return e, b0, lo_mask, [], None
        from ..ops.fingerprint import rabin_rows
        packed = table.rows[:, spec.off:spec.off + spec.length].contiguous()
        e, b0, lo_mask = R.build_keys([rabin_rows(packed)])
        return e, b0, lo_mask, [], (packed, ("bytes", spec.length))
    if kind == "cols":
        cols, skeys = spec, [None] * len(spec)
    else:
        cols, skeys = TR.eq_key_columns(res, table)
    for c in cols:
        if c.dtype not in R.KEY_TYPES or c.dim() != 1:
            raise NotTraceable(f"key dtype {c.dtype}")
    if _wide(cols):
        fp, packed = _wide_key(cols)
        e, b0, lo_mask = R.build_keys([fp])
        return e, b0, lo_mask, skeys, (packed, tuple(str(c.dtype) for c in cols))
    e, b0, lo_mask = R.build_keys(cols)
    return e, b0, lo_mask, skeys, None


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


def _entries_home(bs, n: int, v):
    """Where a producer writes the E64 sort entries of a pitch-128 table: ent_a for the one-rank
    sort; with several ranks the send buffer's first n * 8 bytes ("e64@out": the fine-bucket
    exchange's entry sort then ends in ent_a, away from the rows its pack writes)."""
    if v.world.collective or S.bucket_sort_ok(n, 10):
        # (one rank, bucket sort: its three look-back passes end in ent_a, away from the output)
        return bs.bufs.rows_out.view(-1)[: n * 8].view(torch.int64), "e64@out"
    return bs.bufs.ent_a, "e64"


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
            if v.stage.id in getattr(v.runner, "pitch_gen_stages", ()):
                # only the fused OrderBy reads this table: records at a 128-byte pitch, the sort's
                # E64 entries + window histograms written with them (several ranks: into the send
                # buffer's memory, free until the exchange's pack, see SortBuffers.entry_pair)
                rows = v.alloc_rows(hi - lo, 100, layout="pitch128")
                if rows is not None:
                    t = DeviceTable(hi - lo, Shape("rows", key_off=0, key_len=10), rows=rows)
                    bs = _pooled_set(t, v)
                    rng = torch.tensor([-1, 0], dtype=torch.int64, device=rows.device)
                    ent, fmt = _entries_home(bs, hi - lo, v)
                    TSK.generate_with_keys64_pitch128(bs.bufs.rows_in[: hi - lo], lo, int(q.get("seed", 0)),
                                                      ent, rng, hist=True)
                    bs.keys_ready = (rows.data_ptr(), hi - lo, 0, 10, rng, fmt)
                    return t
            rows = v.alloc_rows(hi - lo, 100)
            t = DeviceTable(hi - lo, Shape("rows", key_off=0, key_len=10), rows=rows)
            bs = _pooled_set(t, v)
            if bs is not None:
                # producer-side key extraction: a following OrderBy(key bytes 0..9) starts sorting
                rng = torch.tensor([-1, 0], dtype=torch.int64, device=rows.device)
                if v.world.size > 1 and v.stage.id in getattr(v.runner, "lazy_gen_stages", ()):
                    # only a fused distributed OrderBy reads this table: nothing is written now;
                    # the sort's send side generates the sample keys, the range partition and the
                    # records (into the send buckets) itself (ops/recordsort.pack_gen), any other
                    # consumer materialises the records first
                    bs.keys_ready = (rows.data_ptr(), hi - lo, 0, 10, None, "gen")
                    bs.lazy_gen = (lo, int(q.get("seed", 0)))
                    return t
                if v.world.size == 1 and S.compact_sort_ok(rows, 10):
                    # one rank: the sort takes the compact 8-byte entries
                    TSK.generate_with_keys64(rows, lo, int(q.get("seed", 0)), bs.bufs.ent_a.view(-1), rng)
                    fmt = "e64"
                else:
                    TSK.generate_with_keys(rows, lo, int(q.get("seed", 0)), bs.bufs.ent_a, rng)
                    fmt = "e128"
                bs.keys_ready = (rows.data_ptr(), hi - lo, 0, 10, rng, fmt)
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
            # the generator's value contract (models/records_cpu.py): keys in [0, nk), payloads
            # mix64(..) >> 33, i.e. 31-bit -- column statistics for operators that pack by width
            # (``bounds=0`` withholds them, as a stored table would: operators then measure them)
            from . import stats
            if str(q.get("bounds", "1")) != "0":
                stats.set_bounds(cols[0], 0, nk - 1)
                for c in cols[1:]:
                    stats.set_bounds(c, 0, (1 << 31) - 1)
            names = FIELDS[:ncols]
            return DeviceTable.from_columns(dict(zip(names, cols)), Shape("tuple", names))
        if kind == "names":
            from ..models import names as NM
            from ..models.records_cpu import dim_multiplier
            nk = int(q.get("keys", 1 << 20))
            return NM.device_table(lo, hi - lo, nk, int(q.get("seed", 0)),
                                   dim_multiplier(nk) if q.get("mode") == "dim" else 0, v.device, NM.namelen(q))
        if kind == "range":
            start = int(q.get("start", 0))
            a = torch.arange(start + lo, start + hi, dtype=torch.int32 if start + hi < 2**31 else torch.int64,
                             device=v.device)
            return DeviceTable.from_columns({"v": a}, Shape("scalar", ["v"]))
    if scheme == "hbm":
        return provider_for(uri).get(uri)["local"][v.partition]
    if scheme == "host":
        from ..io.hosttable import HostRows
        from ..ops.extsort import _copy
        from ..io.hosttable import HostColumns
        b = provider_for(uri).get(uri)["local"].get(v.partition)
        if isinstance(b, HostColumns):
            return b.to_device(v.device)                # pinned host columns -> HBM
        if isinstance(b, HostRows):
            # pinned host tier -> HBM (one DMA; a following OrderBy sorts the pooled rows in place)
            rows = v.alloc_rows(b.n, b.stride)
            _copy(rows, b.rows, None)
            return DeviceTable(b.n, Shape("rows", key_off=b.key_off, key_len=b.key_len), rows=rows)
        t = from_objects(list(b or []), op.get("dtype"), v.device)
        if t is None:
            raise NotTraceable("non-columnar host records")
        return t
    if scheme == "text":
        # raw bytes -> HBM heap -> line (offset, length) pairs on the device
        from ..ops import text as TX
        from .table import text_table
        from .. import types as T
        prov = provider_for(uri)
        if v.device.type == "cuda" and hasattr(prov, "ranges"):
            # the partition's byte range through the native chunked reader (pinned ring -> HBM)
            from ..io import reader as RD
            f, a, b = prov.ranges(uri)[v.partition]
            heap = RD.read_to_device(f, v.device, offset=a, length=b - a)
        else:
            data = prov.read_partition_bytes(uri, v.partition)
            heap = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(v.device) if data else \
                torch.zeros(0, dtype=torch.uint8, device=v.device)
        off, ln = TX.lines(heap)
        t = text_table(heap, off, ln, T.LineRecord)
        t.whole_heap = True           # every line of the heap, in order (tokenise the heap directly)
        return t
    prov = provider_for(uri)
    if scheme in ("partfile", "file") and v.device.type == "cuda":
        from ..io import reader as RD
        rp = prov.rows_part(uri, v.partition)
        if rp is not None:
            # raw fixed-width rows (e.g. an out-of-core sort's output): chunked reader -> pooled HBM
            mm, ko, kl = rp
            stats = getattr(v.runner, "read_stats", None)
            spec = getattr(v.runner, "pitch_gen_stages", {}).get(v.stage.id)
            if spec is not None and mm.shape[1] == 100 and 0 < mm.shape[0] < (1 << 32):
                # only the one-rank OrderBy reads these 100-byte rows: stored at a 128-byte pitch
                # (one aligned HBM line per record) and the sort's compact entries + window
                # histograms extracted from them right after the read, as the generator does
                rows = v.alloc_rows(mm.shape[0], 100, layout="pitch128")
                if rows is not None:
                    n = mm.shape[0]
                    t = DeviceTable(n, Shape("rows", key_off=ko, key_len=kl), rows=rows)
                    RD.read_rows_to_device(mm.filename, v.device, int(mm.offset), n, 100, rows, stats=stats)
                    bs = _pooled_set(t, v)
                    if bs is not None and spec[0] == 0:
                        ent, fmt = _entries_home(bs, n, v)
                        _, part = S.extract_keys64_tile(bs.bufs.rows_in[:n], 0, spec[1], 0, ent, hist=True)
                        S.note_gen_hist(ent[:n], n, part)
                        bs.keys_ready = (rows.data_ptr(), n, 0, spec[1], None, fmt)
                    return t
            rows = v.alloc_rows(mm.shape[0], mm.shape[1])
            if mm.shape[0]:
                RD.read_to_device(mm.filename, v.device, offset=int(mm.offset), length=rows.numel(),
                                  out=rows.view(-1), stats=stats)
            return DeviceTable(mm.shape[0], Shape("rows", key_off=ko, key_len=kl), rows=rows)
        # binary part: bytes -> HBM by the chunked pinned reader -> columns with the device codec
        # (fixed-width records: one thread per field; strings: parallel over the part's record
        # blocks, the part's bytes becoming the string heap)
        from ..ops import codec as CD
        sch = prov.schema(uri) or {}
        dt = op.get("dtype") or sch.get("dtype")
        if sch.get("format", "binary") == "binary" and dt is not None and \
                (CD.layout(dt) is not None or CD.var_layout(dt) is not None):
            path = prov.part_file(uri, v.partition) if hasattr(prov, "part_file") else None
            if path is not None:
                buf = RD.read_to_device(path, v.device)
            else:
                data = prov.read_partition_bytes(uri, v.partition)
                buf = torch.frombuffer(bytearray(data), dtype=torch.uint8).to(v.device) if data else \
                    torch.zeros(0, dtype=torch.uint8, device=v.device)
            if CD.layout(dt) is not None:
                t = CD.decode(buf, dt)
                # column bounds the writer measured (runtime/gpu_executor._commit_partfile_impl)
                from . import stats as GST
                for f, (lo, hi) in (sch.get("bounds") or {}).items():
                    c = t.cols.get(f) if t is not None else None
                    if c is not None and c.dtype in (torch.int64, torch.int32, torch.int16, torch.int8):
                        GST.set_bounds(c, int(lo), int(hi))
            else:
                from ..io import partfile as PF
                idx = PF.read_index(path) if path is not None else None
                t = None
                if idx is not None:
                    n, _nb, blk, offs = idx
                    try:
                        t = CD.decode_var(buf, dt, n, torch.from_numpy(offs).to(v.device), blk)
                    except CD.DecodeError as e:     # a sidecar that does not match the part: rebuilt
                        log.warning("%s: %s; the block index is rebuilt from the part", path, e)
                        idx = None
                if idx is None:
                    n, offs, blk = CD.block_index(buf, dt)
                    t = CD.decode_var(buf, dt, n, offs, blk)
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


def op_sequence_equal(op, inputs, v):
    """SequenceEqual of the two merged inputs (reference SequenceEqual: same length and pairwise
    Equals in order) on the device: the lengths, then every field compared elementwise after
    dtype promotion (NaN != NaN, as Python's ==).  Tables with string heaps or different record
    shapes, and a custom comparer, stay on the host."""
    if op.get("comparer") is not None or len(inputs) != 2:
        raise NotTraceable("SequenceEqual with a comparer")
    a, b = _check(inputs[0]), _check(inputs[1])
    if a.heap is not None or b.heap is not None or a.strs or b.strs:
        raise NotTraceable("SequenceEqual over strings")
    if a.n != b.n:
        return _scalar_table([False], torch.bool, v.device)
    if a.n == 0:
        return _scalar_table([True], torch.bool, v.device)
    if (a.rows is None) != (b.rows is None):
        raise NotTraceable("SequenceEqual of differently laid out tables")
    if a.rows is not None:
        if a.rows.shape[1] != b.rows.shape[1]:
            return _scalar_table([False], torch.bool, v.device)
        eq = torch.equal(a.rows[: a.n], b.rows[: b.n])
        return _scalar_table([bool(eq)], torch.bool, v.device)
    fa, fb = list(a.shape.fields), list(b.shape.fields)
    if a.shape.kind != b.shape.kind or len(fa) != len(fb):
        raise NotTraceable("SequenceEqual of different record shapes")
    ok = torch.ones((), dtype=torch.bool, device=v.device)
    for x, y in zip(fa, fb):
        cx, cy = a.cols[x][: a.n], b.cols[y][: b.n]
        if cx.shape[1:] != cy.shape[1:]:
            return _scalar_table([False], torch.bool, v.device)
        dt = torch.promote_types(cx.dtype, cy.dtype)
        ok = ok & (cx.to(dt) == cy.to(dt)).all()
    return _scalar_table([bool(ok.item())], torch.bool, v.device)


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
    if bs is not None and bs.layout == "pitch128":
        # records at a 128-byte pitch (op_read of a one-rank gen://terasort -> OrderBy stage)
        kind, spec = TR.key_columns(TR.call(op["key"], t), t)
        if op.get("comparer") is None and not op.get("descending", False) and kind == "bytes" and spec.length <= 16:
            kr = bs.take_keys(t.rows, spec.off, spec.length)
            info = {}
            out = S.sort_rows_pitch128(bs.bufs.rows_in[: t.n], bs.bufs.rows_out, bs.bufs.ent_a, spec.off,
                                       spec.length, keys_ready=kr is not None and kr[2] in ("e64", "e64@out"),
                                       stats=info, keys_fmt="e64" if kr is None else kr[2])
            if v.runner is not None:
                v.runner.last_sort_path = info.get("path")
            return DeviceTable(out.shape[0], t.shape, rows=out)
        bs = None                                   # any other sort of such a table: generic path
    if bs is not None and op.get("comparer") is None:
        # in-place key-pointer sort of pooled rows: rows_in -> rows_out, entries in the pool
        kind, spec = TR.key_columns(TR.call(op["key"], t), t)
        if kind == "bytes" and spec.length <= 12:
            kr = bs.take_keys(t.rows, spec.off, spec.length)
            out = RS.local_sort_rows(t.rows, bs.bufs.rows_out, bs.bufs.ent_a, bs.bufs.ent_b, spec.off, spec.length,
                                     descending=op.get("descending", False),
                                     hi_bounds=None if kr is None else kr[:2], keys_ready=kr is not None,
                                     keys_fmt="e128" if kr is None else kr[2])
            return DeviceTable(out.shape[0], t.shape, rows=out)
    _, perm, _ = sort_perm(t, op["key"], op.get("comparer"), op.get("descending", False))
    return t.take(perm)


def hash_keys(table: DeviceTable, key_fn):
    """Key selector -> (HashKey fields, tuple_form) for stable_hash_dest: the key VALUE the host
    partitioner would hash (runtime/vertex_ops.stable_hash), whatever column widths this
    partition inferred."""
    res = TR.call(key_fn, table)

    def field(v):
        if isinstance(v, TR.StrCol):
            return R.HashKey.string(v.heap, v.off, v.len)
        if isinstance(v, TR.ByteField):
            return R.HashKey.bytes_field(table.rows, v.off, v.length)
        c = TR._as_col(v, table.n, table.device)
        if c.dtype not in R.KEY_TYPES or c.dim() != 1:
            raise NotTraceable(f"hash key of dtype {c.dtype}")
        return R.HashKey.column(c)

    if isinstance(res, TR.RowProxy):
        return [R.HashKey.bytes_field(table.rows, 0, table.rows.shape[1])], False
    if isinstance(res, TR.RecProxy):
        sh = table.shape
        if sh.kind == "scalar":
            return [field(TR._field(table, sh.fields[0]))], False
        if sh.kind not in ("tuple", "dataclass"):
            raise NotTraceable(f"hash of a {sh.kind} record")
        items = [TR._field(table, f) for f in sh.fields]
        if len(items) > R.MAX_HASH_COLS:
            raise NotTraceable("record key with more than 8 fields")
        return [field(x) for x in items], True
    if isinstance(res, tuple):
        if not res or len(res) > R.MAX_HASH_COLS:
            raise NotTraceable("tuple key of 0 or more than 8 fields")
        if any(isinstance(x, tuple) for x in res):
            raise NotTraceable("nested tuple key")
        return [field(x) for x in res], True
    return [field(res)], False


def hash_partition_perm(table: DeviceTable, key_fn, n: int):
    """-> (row permutation grouping rows by destination, n+1 port offsets).  The destination is
    the host partitioner's (hash & 0x7FFFFFFF) % n of the key value, so device and host vertices
    of one stage always agree.  n > 256 takes one stable 8-bit pass per destination byte."""
    if n > (1 << 24):
        raise NotTraceable("more than 2^24 hash partitions")
    if table.n >= (1 << 32):
        raise NotTraceable("hash partition of 2^32 rows or more")
    keys, tup = hash_keys(table, key_fn)
    e, _ = R.stable_hash_dest(keys, table.n, n, tup, table.device)
    shift = 64
    while True:
        e, starts = S.partition_pass(e, shift)
        shift += 8
        if n <= (1 << (shift - 64)):
            break
    if n <= 256:
        st = starts[: n + 1]
    else:
        st = torch.searchsorted(e[:, 1].contiguous(), torch.arange(n + 1, dtype=torch.int64, device=e.device))
    return _perm(e), st.tolist()


def _port_order(n: int, world_size: int, place=None):
    """Bucket order of a partition vertex's ports: rank-major for a multi-rank job (port p lives
    on rank ``place[p]``, p % W without a placement), so each destination rank's rows are one
    contiguous slice -> (order, LUT)."""
    if world_size <= 1 or n <= 1:
        return None, None
    rank = (lambda p: place[p]) if place is not None and len(place) >= n else (lambda p: p % world_size)
    order = sorted(range(n), key=lambda p: (rank(p), p))
    if order == list(range(n)):
        return None, None
    lut = [0] * 256
    for i, p in enumerate(order):
        lut[p] = i
    return order, lut


def _dest_place(v):
    r = getattr(v, "runner", None)
    return getattr(r, "place", None)


def partition_by_entries(t: DeviceTable, e: torch.Tensor, n: int, world_size: int = 1, place=None):
    """Port-grouped copy of ``t``: row i goes to port ``e[i, 1]`` (< n <= 256), stable within a
    port, every column moved in one pass (ops/channel.scatter_columns, csrc/kernels/channel.hip).
    None when the table's columns do not fit that kernel."""
    from ..ops import channel as CH
    if n > 256:
        return None
    cols = [t.rows] if t.rows is not None else list(t.cols.values())
    if not cols or not CH.kernel_ok(cols):
        return None
    order, lut = _port_order(n, world_size, place)
    lut_t = torch.tensor(lut, dtype=torch.uint8, device=t.device) if lut is not None else None
    outs, cnt = CH.scatter_columns(e, t.n, cols, lut_t)
    offs = [0]
    for c in cnt[:n].tolist():
        offs.append(offs[-1] + int(c))
    if t.rows is not None:
        nt = DeviceTable(t.n, t.shape, rows=outs[0])
    else:
        nt = DeviceTable(t.n, t.shape, dict(zip(t.cols.keys(), outs)), heap=t.heap, strs=t.strs)
        for k, o in nt.cols.items():           # a permutation of the rows keeps the column bounds
            stats.inherit(o, t.cols[k])
    return Ported(nt, offs, order)


def op_hash_partition(op, inputs, v):
    t = _check(_one(inputs))
    n = op["count"]
    if op.get("comparer") is not None:
        raise NotTraceable("custom comparer")
    if t.n == 0:
        return Ported(t, [0] * (n + 1))
    if n <= 256 and t.n < (1 << 32):
        keys, tup = hash_keys(t, op["key"])
        # one port byte per row (not 16-byte entries): the partition pass reads 1 B/row of
        # destinations and the temporaries of a shuffle shrink by 15 B/row
        e, _ = R.stable_hash_dest(keys, t.n, n, tup, t.device, ports=t.device.type == "cuda")
        out = partition_by_entries(t, e, n, v.world.size, _dest_place(v))
        if out is not None:
            return out
    perm, st = hash_partition_perm(t, op["key"], n)
    return Ported(t.take(perm), st)


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


def _entries_table(t):
    """A sample / separator table of sort entries (the device sample's layout).  A partition whose
    sample ran on the host delivers key values instead: the consumer falls back to the host too."""
    if not isinstance(t, DeviceTable) or "lo" not in t.cols or "hi" not in t.cols:
        raise NotTraceable("sample keys came from the host path")
    return t


def op_separators(op, inputs, v):
    t = _entries_table(_check(_one(inputs)))
    n = op["count"]
    if t.n == 0:
        return DeviceTable.from_columns({"lo": torch.empty(0, dtype=torch.int64, device=v.device),
                                         "hi": torch.empty(0, dtype=torch.int64, device=v.device)}, E_SHAPE)
    e = torch.stack([t.cols["lo"], t.cols["hi"]], 1).contiguous()
    srt = S.sort_entries(e, 0, 128)
    pos = torch.tensor([(j * t.n) // n for j in range(1, n)], dtype=torch.int64, device=e.device)
    s = srt.index_select(0, pos)
    return DeviceTable.from_columns({"lo": s[:, 0].contiguous(), "hi": s[:, 1].contiguous()}, E_SHAPE)


def _separator_entries(t: DeviceTable, key_fn, seps: list) -> torch.Tensor:
    """User range separators (host key values, RangePartition(keySelector, rangeSeparators)) as
    sort entries in the encoding of this partition's key columns, so the device range_dest
    compares them exactly like the host's bisect over the same keys."""
    if len(seps) > 255:
        raise NotTraceable("more than 255 range separators")
    kind, spec = TR.key_columns(TR.call(key_fn, t), t)
    if kind == "bytes":
        if any(not isinstance(x, (bytes, bytearray)) or len(x) != spec.length for x in seps):
            raise NotTraceable("byte-key separators of another length")
        rows = torch.tensor([list(x) for x in seps], dtype=torch.uint8, device=t.device).reshape(len(seps), spec.length)
        return S.extract_keys(rows.contiguous(), 0, spec.length, 0)
    k = len(spec)
    cols = []
    for j, c in enumerate(spec):
        vals = [x[j] if k > 1 else x for x in seps]
        if k > 1 and any(not isinstance(x, tuple) or len(x) != k for x in seps):
            raise NotTraceable("separators do not match the composite key")
        col = torch.tensor(vals, dtype=c.dtype, device=t.device)
        if any(float(a) != float(b) for a, b in zip(vals, col.tolist())):
            raise NotTraceable("separator not representable in the key column type")
        cols.append(col)
    e, _, _ = R.build_keys(cols, [False] * k)
    return e


def op_range_partition(op, inputs, v):
    t = _check(inputs[0])
    n = op["count"]
    seps_t = inputs[1] if len(inputs) > 1 else None
    if t.n == 0:
        return Ported(t, [0] * (n + 1))
    e, _, lo_mask = key_entries(t, op["key"], op.get("comparer"), False)
    if op.get("separators") is not None:
        seps = _separator_entries(t, op["key"], list(op["separators"]))
        S.range_dest(e, seps, lo_mask, descending=op.get("descending", False))
        out = partition_by_entries(t, e, n, v.world.size, _dest_place(v))
        if out is not None:
            return out
        part, starts = S.partition_pass(e, 64)
        return Ported(t.take(_perm(part)), starts[: n + 1].tolist())
    if seps_t is None or seps_t.n == 0:
        return Ported(t, [0] + [t.n] * n)
    seps_t = _entries_table(seps_t)
    seps = torch.stack([seps_t.cols["lo"], seps_t.cols["hi"]], 1).contiguous()
    S.range_dest(e, seps, lo_mask, descending=op.get("descending", False))
    out = partition_by_entries(t, e, n, v.world.size, _dest_place(v))
    if out is not None:
        return out
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
    """Sort by the key columns -> (srt, seg, nseg, rows_at_start, starts).  String keys and keys
    wider than one 96-bit entry are sorted by Rabin-64 fingerprints; every row is then checked
    against its group's representative so a fingerprint collision can never merge two different
    keys (the operator falls back to the host if one ever occurs)."""
    if any(c.dtype not in R.KEY_TYPES or c.dim() != 1 for c in kcols):
        raise NotTraceable("group key of a non-key dtype")
    _row_index_fits(kcols[0].shape[0] if kcols else 0)
    packed = None
    srt = R.int_key_sort(kcols[0]) if len(kcols) == 1 else None
    if srt is not None:
        lo_mask = 0                     # narrow integer key: compact sort, E128 {row, norm key}
    elif _wide(kcols):
        fp, packed = _wide_key(kcols)
        e, b0, lo_mask = R.build_keys([fp])
    else:
        e, b0, lo_mask = R.build_keys(kcols)
    if srt is None:
        srt = S.sort_entries_hybrid(e, b0)
    seg, nseg, starts = R.segment_ids(srt, lo_mask)
    # group representatives straight from the sorted entries (nseg reads); the full row
    # permutation is only materialised when fingerprinted keys must be verified
    rows_at_start = srt[:, 0].index_select(0, starts).bitwise_and_(0xFFFFFFFF)
    verify_str = any(sk is not None for sk in skeys)
    perm = _perm(srt) if (packed is not None or verify_str) else None
    if packed is not None and _rows_differ(packed, perm, packed, rows_at_start.index_select(0, seg)):
        raise NotTraceable("wide key fingerprint collision")
    if verify_str:
        from ..ops.fingerprint import strings_differ
        rep = rows_at_start.index_select(0, seg)          # representative row, in sorted order
        for sk in skeys:
            if sk is not None:
                trip = (sk.heap, sk.off, sk.len)
                if strings_differ(trip, perm, trip, rep):
                    raise NotTraceable("string key fingerprint collision")
    return srt, seg, nseg, rows_at_start, starts


def _key_outputs(kcols, skeys, rows_at_start, srt=None, starts=None):
    """Per-group key columns (string keys keep their heap) -> (cols, strs).  A single int64 key
    is decoded from the sorted entries at the group starts (hi = key ^ sign bit, a near-sequential
    read) instead of a random gather of the key column."""
    out, strs = {}, {}
    if srt is not None and len(kcols) == 1 and skeys[0] is None and kcols[0].dtype == torch.int64:
        out["k0"] = srt[:, 1].index_select(0, starts).bitwise_xor_(-(1 << 63))
        return out, strs
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


_INT_KEYS = (torch.int64, torch.int32, torch.int16, torch.int8, torch.uint8)


def _payload_groups(kcols, skeys, specs, n):
    """R.payload_groups for a single plain integer key on a large partition, else None.  Keys come
    back in the key column's dtype."""
    if len(kcols) != 1 or skeys[0] is not None or kcols[0].dtype not in _INT_KEYS or n < R.PAYLOAD_SORT_MIN_ROWS:
        return None
    k = kcols[0]
    got = R.payload_groups(k.to(torch.int64), specs)
    if got is None or k.dtype == torch.int64:
        return got
    return got[0].to(k.dtype), got[1]


def _radix_groups(kcols, skeys, specs, n, nd=None):
    """(keys, aggregate columns) through ops/radixagg.py for one plain integer key on a large
    partition, else None.  Keys come back in the key column's dtype."""
    from ..ops import radixagg as RA
    if len(kcols) != 1 or skeys[0] is not None or kcols[0].dtype not in _INT_KEYS or not RA.wanted(kcols[0]):
        return None
    k = kcols[0]
    got = RA.radix_aggregate(k, specs, nd_est=nd)
    if got is None or k.dtype == torch.int64:
        return got
    return got[0].to(k.dtype), got[1]


def _dense_groups(kcols, skeys, specs, n):
    """(keys, aggregate columns) through ops/densegroup.py (partition by key bits + LDS tables
    addressed by the low key bits) for one plain integer key whose span needs 13..32 bits and
    integer aggregates that pack with it into 16-byte rows, else None."""
    from ..ops import densegroup as DG
    if len(kcols) != 1 or skeys[0] is not None or kcols[0].dtype not in _INT_KEYS or n < DG.MIN_ROWS:
        return None
    return DG.dense_aggregate(kcols[0], specs)


def _fused_int64_groups(kcols, skeys, specs):
    """(keys, aggregate columns) through R.group_reduce_sorted for one plain int64 key, else None."""
    if not R.FUSED_GROUP_KEYS or len(kcols) != 1 or skeys[0] is not None or kcols[0].dtype != torch.int64:
        return None
    _row_index_fits(kcols[0].shape[0])
    srt = R.int_key_sort(kcols[0])
    if srt is None:
        return None
    return R.group_reduce_sorted(srt, specs, -(1 << 63))


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
    nd_est = None
    if len(kcols) == 1 and skeys[0] is None and not kcols[0].is_floating_point() and t.n >= (1 << 16):
        nd, m = R.estimate_distinct(kcols[0])
        from ..ops.radixagg import distinct_upper_estimate
        nd_est = distinct_upper_estimate(nd, m, t.n)
        if (v.partitions > 1 or op.get("raw_ok")) and op.get("adaptive", True) and nd_est >= RAW_PARTIAL_FRACTION * t.n:
            # almost every key distinct: folding would barely shrink the rows the shuffle moves
            # but cost a full aggregation pass (8-rank GroupBy, 2^30 keys per 1.25e9 rows: 173 vs
            # 104 ms per rank, profiles/r5/gb_lb8_*.log): the rows go out as a raw partial table
            # (``raw_ok``: a streamed GroupBy whose dense running state folds the rows itself)
            return _raw_partial(d, t, kcols[0], form)
        if nd <= R.HASH_AGG_MAX_KEYS and nd * 8 < m:
            got = R.hash_aggregate(kcols[0], specs)
            if got is not None:
                keys, res = got
                out = {"k0": keys}
                for nm, r in zip(names, res):
                    out[nm] = r
                return _partial_table(out, {}, d, 1, form)
    # one integer key over a span of <= 2^32 values: partition by key bits, then LDS tables
    # addressed by the low key bits (no sort, no hash, no gather)
    got = _dense_groups(kcols, skeys, specs, t.n)
    if got is not None:
        out = {"k0": got[0]}
        for nm, r in zip(names, got[1]):
            out[nm] = r
        return _partial_table(out, {}, d, 1, form)
    # one integer key, many distinct keys: radix-partitioned LDS aggregation (no sort, no gather)
    got = _radix_groups(kcols, skeys, specs, t.n, nd_est)
    if got is not None:
        out = {"k0": got[0]}
        for nm, r in zip(names, got[1]):
            out[nm] = r
        return _partial_table(out, {}, d, 1, form)
    # one int64 key: sort through 8-byte entries, then one reduction pass that finds the groups
    # itself (no segment-id array, keys written at the group starts)
    fused = _fused_int64_groups(kcols, skeys, specs)
    if fused is not None:
        out = {"k0": fused[0]}
        for nm, r in zip(names, fused[1]):
            out[nm] = r
        return _partial_table(out, {}, d, 1, form)
    # one int64 key folding <= 3 columns: the values ride in the sort entries (no random gather)
    got = _payload_groups(kcols, skeys, specs, t.n)
    if got is not None:
        out = {"k0": got[0]}
        for nm, r in zip(names, got[1]):
            out[nm] = r
        return _partial_table(out, {}, d, 1, form)
    srt, seg, nseg, rows_at_start, starts = _group_keys(kcols, skeys)
    out, strs = _key_outputs(kcols, skeys, rows_at_start, srt, starts)
    # every aggregate in one fused segmented-reduce pass
    for nm, res in zip(names, R.seg_reduce_multi(srt, seg, nseg, specs)):
        out[nm] = res
    return _partial_table(out, strs, d, len(kcols), form)


def _accumulate_partials(t, d):
    """RecursiveAccumulate over a device partial table: (key values, groups, iterator over the
    per-spec accumulator columns) with one group per distinct key."""
    nkeys = t.shape.pytype.nkeys
    kcols, skeys = TR.eq_key_columns(tuple(TR.Col(v) if isinstance(v, torch.Tensor) else v
                                           for v in _key_values(t, nkeys)), t)
    specs = []
    for j, a in enumerate(d.aggs):
        col = t.cols.get(f"a{j}")
        if a.kind == "count":
            # int8 counts are the ones of a raw partial (_raw_partial; a folded partial's counts are
            # int64, and a mix of both arrives promoted): count the rows instead of summing them,
            # one value column less for the packed aggregation rows
            implicit = col is None or col.dtype == torch.int8
            specs.append(("count", None, torch.int64) if implicit else ("sum", col, torch.int64))
        elif a.kind == "sum":
            specs.append(("sum", col, col.dtype))
        elif a.kind in ("min", "max"):
            specs.append((a.kind, col, col.dtype))
        elif a.kind == "avg":
            c = t.cols.get(f"c{j}")
            specs += [("sum", col, torch.float64),
                      ("count", None, torch.int64) if c is None or c.dtype == torch.int8 else ("sum", c, torch.int64)]
        elif a.kind in ("any", "all"):
            specs.append(("max" if a.kind == "any" else "min", col, torch.int64))
    got = _dense_groups(kcols, skeys, specs, t.n)
    if got is None:
        got = _radix_groups(kcols, skeys, specs, t.n)
    if got is None:
        got = _payload_groups(kcols, skeys, specs, t.n)
    if got is not None:
        return [got[0]], got[0].shape[0], iter(got[1])
    srt, seg, nseg, rows_at_start, starts = _group_keys(kcols, skeys)
    kout, kstrs = _key_outputs(kcols, skeys, rows_at_start, srt, starts)
    keys = _key_values(DeviceTable(nseg, Shape("tuple", list(kout)), kout, strs=kstrs), nkeys)
    return keys, nseg, iter(R.seg_reduce_multi(srt, seg, nseg, specs))


def combine_partials(t, d):
    """Partial tables (concatenated in ``t``) folded into one partial row per distinct key, in the
    same partial layout: the combine step of a streamed GroupBy (runtime/stream_agg.py), whose
    running state stays a partial table until the final reduce."""
    if t.shape.kind != "partial":
        raise NotTraceable("combine_partials: not a device partial table")
    if t.strs:
        raise NotTraceable("combine_partials: string keys")
    if t.n == 0:
        return t
    keys, nseg, res = _accumulate_partials(t, d)
    out = {f"k{i}": k for i, k in enumerate(keys)}
    for j, a in enumerate(d.aggs):
        out[f"a{j}"] = next(res)
        if a.kind == "avg":
            out[f"c{j}"] = next(res)
    m = t.shape.pytype
    meta = PartialMeta(m.nkeys, m.kinds, m.key_form)      # folded: the standard (not raw) layout
    for j, a in enumerate(d.aggs):         # min / max / any / all keep the partial table's dtypes
        col = t.cols.get(f"a{j}")            # (sums and counts stay widened: no overflow on the way)
        if col is not None and out[f"a{j}"].dtype != col.dtype and a.kind in ("min", "max", "any", "all"):
            out[f"a{j}"] = out[f"a{j}"].to(col.dtype)
    tb = DeviceTable.from_columns(out, Shape("partial", list(out), meta))
    return tb


# estimated distinct keys / rows above which a multi-partition GroupBy's partial step ships raw rows
RAW_PARTIAL_FRACTION = 0.5


def _raw_partial(d, t, key, form):
    """A partial table of one row per record, in the standard partial layout: the key column and
    each aggregate's value column as they are, counts as int8 ones (the final step sums them
    into int64; a rank whose partial did fold sends int64 counts and the exchange promotes).
    Ranks may decide differently, so the layout must not differ from a folded partial."""
    out = {"k0": key}
    ones = None
    for j, a in enumerate(d.aggs):
        val = _agg_value(a, t)
        if a.kind in ("count", "avg") and (val is None or a.kind == "avg"):
            if ones is None:
                ones = torch.ones(t.n, dtype=torch.int8, device=t.device)
                stats.set_bounds(ones, 1, 1)
        if a.kind == "count":
            out[f"a{j}"] = ones if val is None else val
        elif a.kind == "avg":
            out[f"a{j}"] = val.to(torch.float64)
            out[f"c{j}"] = ones
        else:
            out[f"a{j}"] = val
    meta = PartialMeta(1, tuple(a.kind for a in d.aggs), form)
    return DeviceTable.from_columns(out, Shape("partial", list(out), meta))


def op_group_final(op, inputs, v):
    t = _check(_one(inputs))
    d = op["decomp"]
    if t.n == 0:
        raise NotTraceable("empty partition")
    if t.shape.kind != "partial":
        raise NotTraceable("group_final input is not a device partial table")
    return final_reduce(t, d)


def final_reduce(t, d):
    """RecursiveAccumulate + FinalReduce of a partial table -> the GroupBy's result table."""
    keys, nseg, res = _accumulate_partials(t, d)
    vals = []
    for j, a in enumerate(d.aggs):
        col = t.cols.get(f"a{j}")
        r = next(res)
        if col is None:                      # a raw partial's implicit count
            vals.append(r)
        elif a.kind in ("count", "sum", "min", "max"):
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
    return _finish_group(d, op_group_partial(dict(op, decomp=d), inputs, v))


def _ordered_group_keys(kcols, skeys):
    """Segments of an input already sorted by the key (K7, OrderedGroupBy): entries in row order,
    groups = runs of equal keys found by adjacent comparison, no sort -> like _group_keys."""
    if any(c.dtype not in R.KEY_TYPES or c.dim() != 1 for c in kcols):
        raise NotTraceable("group key of a non-key dtype")
    _row_index_fits(kcols[0].shape[0] if kcols else 0)
    packed = None
    if _wide(kcols):
        fp, packed = _wide_key(kcols)
        e, _, lo_mask = R.build_keys([fp])
    else:
        e, _, lo_mask = R.build_keys(kcols)
    seg, nseg, starts = R.segment_ids(e, lo_mask)
    rows_at_start = starts
    if packed is not None or any(sk is not None for sk in skeys):
        rep = rows_at_start.index_select(0, seg)
        idx = torch.arange(e.shape[0], device=e.device)
        if packed is not None and _rows_differ(packed, idx, packed, rep):
            raise NotTraceable("wide key fingerprint collision")
        from ..ops.fingerprint import strings_differ
        for sk in skeys:
            if sk is not None and strings_differ((sk.heap, sk.off, sk.len), idx, (sk.heap, sk.off, sk.len), rep):
                raise NotTraceable("string key fingerprint collision")
    return e, seg, nseg, rows_at_start, starts


def op_ordered_group_by(op, inputs, v):
    """OrderedGroupBy (reference DryadLinqVertex.cs:586-760): the partition is sorted by the key,
    so every group is a run: one adjacent-difference pass + one segmented reduction."""
    d = op.get("decomp")
    if d is None or op.get("elem") is not None:
        raise NotTraceable("non-decomposable GroupBy")
    t = _check(_one(inputs))
    if op.get("comparer") is not None or any(a.kind not in _GPU_AGGS for a in d.aggs):
        raise NotTraceable("aggregate not supported on the device")
    if t.n == 0:
        raise NotTraceable("empty partition")
    kcols, skeys, form = _key_cols(t, op["key"])
    specs, names = _group_specs(d, t)
    srt, seg, nseg, rows_at_start, starts = _ordered_group_keys(kcols, skeys)
    out, strs = _key_outputs(kcols, skeys, rows_at_start, srt, starts)
    for nm, res in zip(names, R.seg_reduce_multi(srt, seg, nseg, specs)):
        out[nm] = res
    return _finish_group(d, _partial_table(out, strs, d, len(kcols), form))


def _finish_group(d, tb):
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
    if op.get("comparer") is not None:
        raise NotTraceable("custom comparer")
    if t.n <= 1:
        return t
    e, b0, lo_mask, packed = _record_entries(t)
    srt = S.sort_entries_hybrid(e, b0)
    seg, _, starts = R.segment_ids(srt, lo_mask)
    _verify_segments(packed, srt, seg, starts)
    return t.take(_perm(srt).index_select(0, starts))


def _record_entries(t):
    """Whole-record keys for Distinct / set operations -> (entries, begin_bit, lo_mask, packed):
    records up to 96 bits (rows up to 12 bytes) are their own sort key; wider fixed-width records
    are keyed by the Rabin-64 fingerprint of their packed bytes (``packed`` is returned for the
    byte-for-byte segment check)."""
    if t.heap is not None or t.strs:
        raise NotTraceable("records with string fields")
    if t.rows is not None:
        if t.rows.shape[1] <= 12:
            e, b0, lm = key_entries(t, lambda r: r[0:t.rows.shape[1]])
            return e, b0, lm, None
        packed = t.rows.contiguous()
    else:
        cols = [t.cols[f] for f in t.shape.fields]
        if all(c.dim() == 1 and c.dtype in R.KEY_TYPES for c in cols) and not _wide(cols):
            e, b0, lm = R.build_keys(cols)
            return e, b0, lm, None
        packed = torch.cat([(c + 0.0 if c.is_floating_point() else c).contiguous().view(torch.uint8)
                            .reshape(t.n, -1) for c in cols], 1).contiguous()
    from ..ops.fingerprint import rabin_rows
    e, b0, lm = R.build_keys([rabin_rows(packed)])
    return e, b0, lm, packed


def _verify_segments(packed, srt, seg, starts):
    """NotTraceable if two different records share a fingerprint segment."""
    if packed is None:
        return
    perm = _perm(srt)
    if _rows_differ(packed, perm, packed, perm.index_select(0, starts).index_select(0, seg)):
        raise NotTraceable("record fingerprint collision")


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
    e, b0, lo_mask, packed = _record_entries(both)
    srt = S.sort_entries_hybrid(e, b0)
    seg, nseg, starts = R.segment_ids(srt, lo_mask)
    _verify_segments(packed, srt, seg, starts)
    first = _perm(srt).index_select(0, starts)
    if kind == "union":
        return both.take(first)
    side = (torch.arange(both.n, device=both.device) >= a.n).to(torch.int64)   # 0 = left, 1 = right
    lo_side, hi_side = R.seg_reduce_multi(srt, seg, nseg, [("min", side, torch.int64), ("max", side, torch.int64)])
    keep = (lo_side == 0) & (hi_side == 1) if kind == "intersect" else (hi_side == 0)
    return both.take(first[keep])


def op_union(op, inputs, v):
    return _set_op("union", op, inputs)


def op_ordered_distinct(op, inputs, v):
    """Distinct of a partition sorted by the record: keep the first of every run (no sort)."""
    t = _check(_one(inputs))
    if op.get("comparer") is not None:
        raise NotTraceable("custom comparer")
    if t.n <= 1:
        return t
    e, _, lo_mask, packed = _record_entries(t)
    seg, _, starts = R.segment_ids(e, lo_mask)
    _verify_segments(packed, e, seg, starts)
    return t.take(starts)


def _ordered_set(kind, op, inputs):
    """Ordered set operations: the device set operation emits records in ascending key order,
    which is the order the planner promised for ascending, non-fingerprinted records."""
    if op.get("descending"):
        raise NotTraceable("descending ordered set operation")
    a = _check(inputs[0])
    cols = [a.cols[f] for f in a.shape.fields] if a.rows is None else []
    if a.rows is not None and a.rows.shape[1] > 12 or a.rows is None and (_wide(cols) or any(
            c.dim() != 1 or c.dtype not in R.KEY_TYPES for c in cols)):
        raise NotTraceable("fingerprinted records: key order is not record order")
    return _set_op(kind, op, inputs)


def op_ordered_union(op, inputs, v):
    return _ordered_set("union", op, inputs)


def op_ordered_intersect(op, inputs, v):
    return _ordered_set("intersect", op, inputs)


def op_ordered_except(op, inputs, v):
    return _ordered_set("except", op, inputs)


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


def _join_pairs(op, outer, inner, hashed):
    """(outer_row, inner_row, per-outer match counts) of equal keys.  ``hashed``: device hash
    table on the inner keys probed in outer row order (hashjoin.hip: LINQ Join order); else
    radix-sorted entries + merge-path ranges (key order).  Pairs matched through fingerprints
    (string / wide keys) are verified byte for byte."""
    if op.get("comparer") is not None:
        raise NotTraceable("custom comparer")
    eo, b0, lm, so_keys, wo = eq_key_entries(outer, op["outer_key"])
    ei, b1, lm2, si_keys, wi = eq_key_entries(inner, op["inner_key"])
    if (b0, lm) != (b1, lm2) or [k is None for k in so_keys] != [k is None for k in si_keys] or \
            (wo is None) != (wi is None) or (wo is not None and wo[1] != wi[1]):
        raise NotTraceable("join keys of different types")
    if hashed:
        oo, ii, cnt = R.hash_join_pairs(eo, ei, lm)
    else:
        so = S.sort_entries_hybrid(eo, b0)
        si = S.sort_entries_hybrid(ei, b0)
        oo, ii, cnt = R.merge_join_pairs(so, si, lm)
    if oo.shape[0]:
        from ..ops.fingerprint import strings_differ
        for a, b in zip(so_keys, si_keys):
            if a is not None and strings_differ((a.heap, a.off, a.len), oo, (b.heap, b.off, b.len), ii):
                raise NotTraceable("string key fingerprint collision")
        if wo is not None and _rows_differ(wo[0], oo, wi[0], ii):
            raise NotTraceable("wide key fingerprint collision")
    return oo, ii, cnt


def _join(op, inputs, hashed):
    outer, inner = _check(inputs[0]), _check(inputs[1])
    if outer.n == 0 or inner.n == 0:
        raise NotTraceable("empty join side: output type unknown")
    oo, ii, _ = _join_pairs(op, outer, inner, hashed)
    if oo.shape[0] == 0:
        raise NotTraceable("empty join result")
    a, b = outer.take(oo), inner.take(ii)
    return _result_table(_traced(op["result"], TR.proxy(a), TR.proxy(b)), a)


# the hash table wins while the build side stays small (tools/microbench_ops.py, 2^28 probe rows:
# 2^16 build rows hash 14 ms vs sort-merge 22 ms, 2^22 rows 30 vs 29 ms, 2^26 rows 46 vs 40 ms;
# 2^27 x 2^27 rows 38 vs 27 ms): past this many inner rows both sides are sorted instead
HASH_JOIN_MAX_INNER = 1 << 22


def op_hash_join(op, inputs, v):
    """Join (K8; reference HashJoin DryadLinqVertex.cs:852-897): a device hash table on the inner
    keys, probed in outer row order (csrc/kernels/hashjoin.hip: LINQ Join order), or, past
    HASH_JOIN_MAX_INNER inner rows, a sort-merge join (pairs then come in key order)."""
    outer, inner = inputs[0], inputs[1]
    big = isinstance(inner, DeviceTable) and isinstance(outer, DeviceTable) and inner.n > HASH_JOIN_MAX_INNER
    return _join(op, inputs, not big)


def op_merge_join(op, inputs, v):
    """Join of key-ordered inputs (K9; reference MergeJoin DryadLinqVertex.cs:898-1070)."""
    return _join(op, inputs, False)


def op_hash_group_join(op, inputs, v):
    """GroupJoin whose result selector only folds the group with decomposable aggregates
    (Count / Sum / Min / Max / Average / Any / All; reference HashGroupJoin DryadLinqVertex.cs:
    1071-1116): hash-join pairs in outer row order -> per-outer-row segmented reductions over the
    matched inner rows -> the result template evaluated over the outer records' columns."""
    from ..compiler.decomposition import decompose
    outer, inner = _check(inputs[0]), _check(inputs[1])
    if outer.n == 0 or inner.n == 0:
        raise NotTraceable("empty GroupJoin side")
    d = decompose(op["result"])
    if d is None or any(a.kind not in ("count", "sum", "min", "max", "avg", "any", "all") for a in d.aggs):
        raise NotTraceable("GroupJoin result selector does not decompose into device aggregates")
    oo, ii, cnt = _join_pairs(op, outer, inner, True)
    if any(a.kind in ("min", "max", "avg") for a in d.aggs) and bool((cnt == 0).any()):
        raise NotTraceable("Min / Max / Average over an empty group")
    specs, plan = [], []
    for a in d.aggs:
        val = _agg_value(a, inner)
        if a.kind == "count" and val is None:
            plan.append(("count", None))
            continue
        if a.kind in ("count", "any", "all"):
            specs.append(("sum", val, torch.int64))
        elif a.kind == "avg":
            specs.append(("sum", val, torch.float64))
        else:
            specs.append((a.kind, val, val.dtype))
        plan.append((a.kind, len(specs) - 1))
    ent = torch.stack([ii, torch.zeros_like(ii)], 1).contiguous()
    red = R.seg_reduce_multi(ent, oo, outer.n, specs) if specs else []
    vals = []
    for kind, j in plan:
        r = cnt if j is None else red[j]
        if kind == "avg":
            r = r / cnt.to(torch.float64)
        elif kind == "any":
            r = r > 0
        elif kind == "all":
            r = r == cnt
        vals.append(r)
    env = {"key": TR.proxy(outer), "aggs": [TR.Col(x) for x in vals]}
    try:
        res = substitute(d.template, env)
    except NotTraceable:
        raise
    except Exception as ex:  # noqa: BLE001
        raise NotTraceable(f"result template: {ex}")
    return _result_table(res, outer)


op_merge_group_join = op_hash_group_join


# ---------------------------------------------------------------------------------------------
# aggregates (K11): the partial of every partition is ONE pass of the reduce kernel over its HBM
# columns (ops/reduce.py, csrc/kernels/reduce.hip); partials are host scalars in the object
# path's format, so the final vertex (one value per partition) folds them with the object code
_EMPTY_PARTIAL = {"Count": 0, "Sum": 0, "Average": (0, 0), "Any": False, "All": True, "Contains": False,
                  "First": (False, None), "FirstOrDefault": (False, None), "Last": (False, None),
                  "LastOrDefault": (False, None), "Single": (0, None), "SingleOrDefault": (0, None)}


def _agg_column(sel, t):
    """The numeric column an aggregate folds: the records themselves or the traced selector."""
    if sel is None:
        if t.shape.kind != "scalar":
            raise NotTraceable("aggregate over non-scalar records")
        c = t.cols[t.shape.fields[0]]
    else:
        r = TR.call(sel, t)
        if not isinstance(r, TR.Col):
            raise NotTraceable("aggregate selector must produce a numeric field")
        c = r.t.expand(t.n) if r.t.dim() == 0 else r.t
    if c.dim() != 1 or c.is_complex():
        raise NotTraceable("aggregate over a non-scalar field")
    return c


def _record_at(t, i):
    return t.slice(i, i + 1).to_objects()[0]


def op_agg_partial(op, inputs, v):
    from ..ops import reduce as RD
    from ..runtime.vertex_ops import _NONE
    t = _check(_one(inputs))
    s = op["spec"]
    k = s["kind"]
    if s.get("comparer") is not None:
        raise NotTraceable("custom comparer")
    if k not in _EMPTY_PARTIAL and k not in ("Min", "Max"):
        raise NotTraceable(f"{k} with a user accumulator runs on the host")
    n, dev = t.n, t.device
    if n == 0:
        return [_NONE if k in ("Min", "Max") else _EMPTY_PARTIAL[k]]
    pred = s.get("predicate")
    mask = TR.to_mask(TR.call(pred, t), t) if pred is not None else None
    if k == "Count":
        return [n if mask is None else RD.reduce_multi(n, [(RD.COUNT, None, mask)], dev)[0]]
    if k in ("Any", "All"):
        c = n if mask is None else RD.reduce_multi(n, [(RD.COUNT, None, mask)], dev)[0]
        return [c > 0] if k == "Any" else [c == n]
    if k in ("Sum", "Average", "Min", "Max"):
        col = _agg_column(s.get("selector"), t)
        rop = {"Sum": RD.SUM, "Average": RD.SUM, "Min": RD.MIN, "Max": RD.MAX}[k]
        r = RD.reduce_multi(n, [(rop, col, None)], dev)[0]
        if k == "Average":
            return [(r, n)]
        return [bool(r) if col.dtype == torch.bool and k != "Sum" else r]
    if k == "Contains":
        val = s.get("value")
        if t.shape.kind != "scalar" or isinstance(val, bool) or not isinstance(val, (int, float)):
            raise NotTraceable("Contains of a non-numeric value")
        hit = t.cols[t.shape.fields[0]] == val
        return [RD.reduce_multi(n, [(RD.COUNT, None, hit)], dev)[0] > 0]
    if k.startswith("First") or k.startswith("Last"):
        first = k.startswith("First")
        i = (0 if first else n - 1) if mask is None else \
            RD.reduce_multi(n, [(RD.FIRST if first else RD.LAST, None, mask)], dev)[0]
        return [(False, None)] if i is None else [(True, _record_at(t, i))]
    # Single / SingleOrDefault: the number of matches and the first one
    c, i = (n, 0) if mask is None else RD.reduce_multi(n, [(RD.COUNT, None, mask), (RD.FIRST, None, mask)], dev)
    return [(c, _record_at(t, i) if c else None)]


class _AccFold:
    """Symbolic accumulator of a user ``Aggregate(seed, func)``: tracing ``func(acc, x)`` with
    ``acc`` bound to this object records ``acc + T(x)`` (or ``acc - T(x)``, ``T(x) + acc``, ``acc
    + T(x) + c``, ...), or a bitwise fold ``acc ^ T(x)`` / ``acc | T(x)`` / ``acc & T(x)`` of
    integers (checksums, flag unions).  Such a fold is ``seed OP reduce_i T(x_i)`` (the operators
    are associative and commutative), so the sequential vertex becomes one device reduction.  Any
    other use of ``acc`` (products, comparisons, branches, attribute access, mixed operators) is
    not such a fold and raises NotTraceable."""
    __slots__ = ("term", "kind")

    def __init__(self, term=0, kind="sum"):
        self.term, self.kind = term, kind

    @staticmethod
    def _operand(o):
        if isinstance(o, _AccFold):
            raise NotTraceable("accumulator used twice in the fold step")
        return o if isinstance(o, (TR.Col, int, float)) else TR.Col(o)

    def __add__(self, o):
        if self.kind != "sum":
            raise NotTraceable("mixed fold operators")
        return _AccFold(self.term + self._operand(o))

    __radd__ = __add__

    def __sub__(self, o):
        if self.kind != "sum":
            raise NotTraceable("mixed fold operators")
        return _AccFold(self.term - self._operand(o))

    def _bitwise(self, o, kind):
        if self.kind != "sum" or not (isinstance(self.term, int) and self.term == 0):
            raise NotTraceable("mixed fold operators")
        return _AccFold(self._operand(o), kind)

    def __xor__(self, o):
        return self._bitwise(o, "xor")

    def __or__(self, o):
        return self._bitwise(o, "or")

    def __and__(self, o):
        return self._bitwise(o, "and")

    __rxor__, __ror__, __rand__ = __xor__, __or__, __and__

    def __getattr__(self, name):
        raise NotTraceable(f"accumulator used as {name}: not a sum fold")

    def __bool__(self):
        raise NotTraceable("branch on the accumulator")

    def _no(self, *a):
        raise NotTraceable("accumulator in a non-additive expression")

    __mul__ = __rmul__ = __rsub__ = __truediv__ = __rtruediv__ = __floordiv__ = __mod__ = __pow__ = _no
    __lt__ = __le__ = __gt__ = __ge__ = __eq__ = __ne__ = __neg__ = _no
    __hash__ = None


def _bitwise_reduce(col: torch.Tensor, kind: str) -> int:
    """XOR / OR / AND of an integer column by halving folds (log2(n) passes over shrinking
    halves: about two reads of the column)."""
    fn = {"xor": torch.bitwise_xor, "or": torch.bitwise_or, "and": torch.bitwise_and}[kind]
    x = col.to(torch.int64)
    while x.numel() > 1:
        h = x.numel() // 2
        y = fn(x[:h], x[h: 2 * h])
        x = torch.cat([y, x[2 * h:]]) if x.numel() % 2 else y
    return int(x[0].item())


def op_aggregate_seq(op, inputs, v):
    """Non-associative ``Aggregate(seed, func[, result])`` on the merged partition
    (reference: DryadLinqQueryGen Aggregate without [Associative] runs as one vertex folding the
    whole input, DryadLinqQueryGen.cs:3384-3395).  When ``func`` traces to ``acc + T(x)`` the fold
    is ``seed + sum(T(x))``: one device reduction instead of a host loop over every record.
    Integer folds are exact (a fold that could leave the int64 range, judged from the column's
    min / max, runs on the host with Python ints); float folds are re-associated like ``Sum``.  Without a
    seed the first record seeds the fold (scalar records only)."""
    from ..ops import reduce as RD
    from ..query import _NOSEED
    t = _check(_one(inputs))
    s = op["spec"]
    if t.n == 0:
        raise NotTraceable("empty partition")
    seed = s.get("seed", _NOSEED)
    rows = t
    if seed is _NOSEED:
        if t.shape.kind != "scalar" or t.heap is not None or t.strs or t.shape.fields[0] not in t.cols:
            raise NotTraceable("seedless Aggregate over non-numeric records")
        first = t.cols[t.shape.fields[0]][:1].tolist()[0]
        if isinstance(first, bool) or not isinstance(first, (int, float)):
            raise NotTraceable("seedless Aggregate over non-numeric records")
        if t.n == 1:
            r = s.get("result_selector")
            return [r(first) if r else first]
        rows, seed = t.slice(1, t.n), first
    elif isinstance(seed, bool) or not isinstance(seed, (int, float)):
        raise NotTraceable("non-numeric Aggregate seed")
    res = _traced(s["func"], _AccFold(), TR.proxy(rows))
    if isinstance(res, TR.Col) and isinstance(res.t, _AccFold):     # T(x) + acc via a tensor operand
        res = res.t
    if not isinstance(res, _AccFold):
        raise NotTraceable("Aggregate step is not acc + f(x)")
    term = res.term
    if res.kind != "sum":
        # bitwise fold of integers: seed OP (T(x_1) OP ... OP T(x_n)) (Python ints: exact as long as
        # the seed and the terms are int64 values)
        if isinstance(seed, float) or (isinstance(term, TR.Col) and not isinstance(term.t, torch.Tensor)):
            raise NotTraceable("bitwise Aggregate of non-integers")
        if isinstance(term, bool) or isinstance(term, float):
            raise NotTraceable("bitwise Aggregate of non-integers")
        if isinstance(term, int):
            col = torch.full((rows.n,), term, dtype=torch.int64, device=t.device)
        else:
            col = term.t.expand(rows.n) if term.t.dim() == 0 else term.t
            if col.dim() != 1 or col.is_floating_point() or col.is_complex():
                raise NotTraceable("bitwise Aggregate of non-integers")
        if not -(1 << 63) <= int(seed) < (1 << 63):
            raise NotTraceable("Aggregate seed past int64")
        red = _bitwise_reduce(col[: rows.n].contiguous(), res.kind)
        acc = {"xor": int(seed) ^ red, "or": int(seed) | red, "and": int(seed) & red}[res.kind]
        r = s.get("result_selector")
        return [r(acc) if r else acc]
    if isinstance(term, (int, float)) and not isinstance(term, bool):
        acc = seed + term * rows.n
    else:
        if not isinstance(term, TR.Col) or not isinstance(term.t, torch.Tensor):
            raise NotTraceable("Aggregate term is not a numeric field")
        col = term.t.expand(rows.n) if term.t.dim() == 0 else term.t
        if col.dim() != 1 or col.is_complex():
            raise NotTraceable("Aggregate term is not a scalar field")
        if col.dtype == torch.bool:
            col = col.to(torch.int64)
        if not col.is_floating_point():
            # the host fold uses Python ints: refuse a device sum that could wrap past int64
            mn, mx = RD.reduce_multi(rows.n, [(RD.MIN, col.contiguous(), None), (RD.MAX, col.contiguous(), None)],
                                     t.device)
            lim = (1 << 63) - 1 - abs(int(seed))
            if max(abs(int(mn)), abs(int(mx))) * rows.n > lim:
                raise NotTraceable("integer Aggregate could overflow int64 on the device")
        acc = seed + RD.reduce_multi(rows.n, [(RD.SUM, col.contiguous(), None)], t.device)[0]
    r = s.get("result_selector")
    return [r(acc) if r else acc]


def _host_partials(inputs) -> list:
    out = []
    for x in inputs:
        if isinstance(x, DeviceTable):
            out.extend(x.to_objects())
        elif isinstance(x, list):
            out.extend(x)
    return out


def op_agg_final(op, inputs, v):
    """Fold the per-partition partials (one host value per partition, the reference's final
    aggregate vertex) with the object implementation; device-table partials are read back."""
    from ..runtime import vertex_ops as VO
    return VO.op_agg_final(op, [_host_partials(inputs)], v)


def op_agg_combine(op, inputs, v):
    """Aggregation-tree interior vertex: partials in, one partial out (object implementation)."""
    from ..runtime import vertex_ops as VO
    return VO.op_agg_combine(op, [_host_partials(inputs)], v)


# ---------------------------------------------------------------------------------------------
# Zip / SelectMany / SlidingWindow / keyed Fork on traced columns
def _traced(fn, *args):
    try:
        return fn(*args)
    except NotTraceable:
        raise
    except (TypeError, AttributeError, RuntimeError, IndexError, ValueError) as e:
        raise NotTraceable(f"{type(e).__name__}: {e}")


def _result_table(res, proto):
    """TR.to_table, except that a record proxy stands for its own table."""
    if isinstance(res, (TR.RecProxy, TR.RowProxy)):
        return object.__getattribute__(res, "_t")
    if isinstance(res, TR.ByteField):
        raise NotTraceable("byte-string projection of a proxied row")
    return TR.to_table(res, proto)


def op_zip(op, inputs, v):
    a, b = _check(inputs[0]), _check(inputs[1])
    n = min(a.n, b.n)
    if n == 0:
        raise NotTraceable("empty Zip input: output type unknown")
    a, b = a.slice(0, n), b.slice(0, n)
    return _result_table(_traced(op["fn"], TR.proxy(a), TR.proxy(b)), a)


def _interleave(tabs):
    """Tables t_0..t_{L-1} of n rows -> n * L rows t_0[0], t_1[0], .., t_0[1], .. (SelectMany order)."""
    t0, L = tabs[0], len(tabs)
    if any(t.heap is not None or t.strs for t in tabs):
        raise NotTraceable("SelectMany over string fields")
    if t0.rows is not None:
        if any(t.rows is None or t.rows.shape[1] != t0.rows.shape[1] for t in tabs):
            raise NotTraceable("SelectMany elements of different layouts")
        return DeviceTable(t0.n * L, t0.shape, rows=torch.stack([t.rows for t in tabs], 1).reshape(t0.n * L, -1))
    for t in tabs[1:]:
        if t.rows is not None or t.shape.kind != t0.shape.kind or t.shape.fields != t0.shape.fields or \
                t.shape.pytype is not t0.shape.pytype or \
                any(t.cols[k].shape[1:] != c.shape[1:] or t.cols[k].is_floating_point() != c.is_floating_point()
                    for k, c in t0.cols.items()):
            raise NotTraceable("SelectMany elements of different layouts")
    # [x, x + 1]: an Int32 field and its int64 arithmetic share the wider type (Python ints)
    wide = {k: functools.reduce(torch.promote_types, [t.cols[k].dtype for t in tabs]) for k in t0.cols}
    cols = {k: torch.stack([t.cols[k].to(wide[k]) for t in tabs], 1).reshape((t0.n * L,) + tuple(c.shape[1:]))
            for k, c in t0.cols.items()}
    return DeviceTable(t0.n * L, t0.shape, cols)


def op_select_many(op, inputs, v):
    """SelectMany whose selector returns a fixed-length list / tuple of traced values: every
    element is a column table, interleaved in record order (one stack per field)."""
    t = _check(_one(inputs))
    if t.n == 0:
        raise NotTraceable("empty partition: output type unknown")
    res = TR.call(op["fn"], t)
    if not isinstance(res, (list, tuple)) or hasattr(res, "_fields") or not res:
        raise NotTraceable("SelectMany selector must return a fixed-length list of traced values")
    r = op.get("result")
    x = TR.proxy(t)
    return _interleave([_result_table(_traced(r, x, e) if r is not None else e, t) for e in res])


def op_sliding_window(op, inputs, v):
    """SlidingWindow(f, w): f sees a list of w proxies over shifted slices of the partition."""
    t = _check(_one(inputs))
    w = int(op["window"])
    m = t.n - w + 1
    if m <= 0:
        raise NotTraceable("window longer than the input: output type unknown")
    wins = [TR.proxy(t.slice(j, j + m)) for j in range(w)]
    return _result_table(_traced(op["fn"], wins), t.slice(0, m))


def op_fork(op, inputs, v):
    """Keyed Fork (IKeyedMultiQueryable): one stable pass routes each record to the port of its
    key (a repeated key routes to its last index, like the object path's dict)."""
    t = _check(_one(inputs))
    keys = op.get("keys")
    if keys is None:
        return _fork_tuple(op, t)
    if t.n == 0:
        raise NotTraceable("empty partition")
    if any(isinstance(k, bool) or not isinstance(k, (int, float)) for k in keys):
        raise NotTraceable("non-numeric fork keys")
    kc = TR.call(op["mapper"], t)
    if not isinstance(kc, TR.Col):
        raise NotTraceable("fork key must be a scalar field")
    col = kc.t.expand(t.n) if kc.t.dim() == 0 else kc.t
    K = len(keys)
    dest = torch.full((t.n,), K, dtype=torch.int64, device=t.device)
    for i, k in enumerate(keys):
        dest.masked_fill_(col == k, i)
    order = torch.argsort(dest, stable=True)
    counts = torch.bincount(dest, minlength=K + 1)[:K].tolist()
    offs = [0]
    for c in counts:
        offs.append(offs[-1] + c)
    return Ported(t.take(order), offs)


def _fork_tuple(op, t):
    """Per-record ForkTuple mapper (reference ForkTuple.cs / DryadLinqEnumerable Fork): the mapper
    is traced once over the partition; port k holds ``Value`` of slot k (a traced field or record)
    for the records whose ``HasValue`` is true, in record order.  Ports may differ in record type,
    so the output is one table per port (PortTables); an unused slot is an empty port."""
    from ..types import ForkTuple, ForkValue
    if not op.get("per_record"):
        raise NotTraceable("ForkTuple mapper over the whole sequence runs on the host")
    if t.n == 0:
        raise NotTraceable("empty partition")
    res = TR.call(op["mapper"], t)
    if not isinstance(res, ForkTuple):
        raise NotTraceable("Fork mapper did not return a ForkTuple")
    tables = []
    for fv in (res.First, res.Second, res.Third):
        if not isinstance(fv, ForkValue):
            raise NotTraceable("ForkTuple slot is not a ForkValue")
        hv = fv.HasValue
        if hv is False or (isinstance(hv, TR.Col) and hv.t.dim() == 0 and not bool(hv.t)):
            tables.append([])
            continue
        tab = _result_table(_traced(lambda: fv.Value), t)
        if hv is True:
            tables.append(tab)
            continue
        if not isinstance(hv, TR.Col) or hv.t.dtype != torch.bool:
            raise NotTraceable("ForkValue.HasValue must be a bool or a boolean field")
        tables.append(tab if hv.t.dim() == 0 else tab.mask(hv.t))
    return PortTables(tables)


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

"""Bounded (chunk-streamed) execution of record-wise stages on the GPU executor.

In the reference every vertex reads its input channel as a stream of buffers and writes its
output channel the same way (RChannelReader / RChannelWriter, DryadVertex/VertexHost/system/
channel/include/channelinterface.h:212-399; the buffer FIFO of channelfifo.h), so a vertex never
holds a whole partition.  The GPU executor's default edge is a whole HBM-resident partition (a
device table is what the next operator's kernels take), which bounds a partition by HBM.

A stage whose program is ``read -> record-wise operators -> write`` does not need that: each
record's output depends on that record only.  Such a stage runs here as a loop over bounded
chunks of its source partition (rows of a stored part through the chunked reader, or a generator
sub-range), each chunk going through the operators on the device and straight into the native
part writer (HBM -> pinned ring -> pwrite threads).  The partition then needs HBM for about two
chunks, not for the partition, and reads, kernels and writes of neighbouring chunks overlap.

Chosen when the source partition is larger than ``StreamChunkBytes`` (context property; default
4 GB) or ``StreamStages=True``.  Record-wise operators: Select, Where, SelectMany (no index
overloads: those need the partition-global record index).
"""
from __future__ import annotations

import os

import torch

from ..gpu.table import DeviceTable, Shape
from ..io.providers import parse_uri, provider_for
from ..utils.log import get_logger

log = get_logger("streaming")

STREAM_OPS = {"select", "where", "select_many", "identity"}
DEFAULT_CHUNK_BYTES = 4 << 30


def _source(runner, s):
    """(kind, info) of a chunkable source of stage s, or None."""
    op = s.ops[0]
    if op["op"] != "read":
        return None
    uri = op["uri"]
    scheme, path, q = parse_uri(uri)
    if scheme == "gen":
        kind = path.strip("/")
        if kind in ("terasort", "records64", "range", "names"):
            return kind, dict(q=q, uri=uri)
        return None
    if scheme == "host":
        # the pinned host tier: row tables (an out-of-core sort's output) and column tables (a
        # streamed result), read back chunk by chunk
        from ..io.hosttable import HostColumns, HostRows
        prov = provider_for(uri)
        if not prov.exists(uri):
            return None
        local = prov.get(uri)["local"]
        if local and all(isinstance(v, HostRows) for v in local.values()):
            return "hostrows", dict(uri=uri, local=local)
        if local and all(isinstance(v, HostColumns) for v in local.values()):
            return "hostcols", dict(uri=uri, local=local)
        return None
    if scheme in ("partfile", "file"):
        prov = provider_for(uri)
        sch = prov.schema(uri) or {}
        if sch.get("format") == "rows":
            return "rows", dict(uri=uri, prov=prov)
        from ..ops import codec as CD
        dt = op.get("dtype") or sch.get("dtype")
        if sch.get("format", "binary") == "binary" and dt is not None and CD.layout(dt) is not None:
            return "fixed", dict(uri=uri, prov=prov, dtype=dt, width=CD.layout(dt)[1])
    return None


def _partition_bytes(kind, info, p) -> int:
    if kind in ("hostrows", "hostcols"):
        v = info["local"].get(p)
        return v.nbytes if v is not None else 0
    if kind in ("rows", "fixed"):
        from ..io import partfile as PF
        m = PF.read_meta(parse_uri(info["uri"])[1])
        return m.parts[p].size if p < m.count else 0
    from ..io.providers import GenProvider
    lo, hi = GenProvider().bounds(info["uri"], p)
    per = {"terasort": 100, "records64": 8 * int(info["q"].get("cols", 8)), "range": 8, "names": 32}[kind]
    return (hi - lo) * per


def streamable(runner, s):
    """The stage's chunk plan (source kind, info, chunk bytes) if it can stream, else None."""
    if not runner.gpu_ok or s.inputs or len(s.ops) < 2 or s.ops[-1]["op"] != "output" or not s.is_output:
        return None
    if any(o["op"] not in STREAM_OPS for o in s.ops[1:-1]):
        return None
    scheme = parse_uri(s.output["uri"])[0]
    if scheme not in ("partfile", "file") or runner.ctx.OutputDataCompressionScheme.value != 0:
        return None
    if s.id in runner.skipped or s.id in runner.gang_stages:
        return None
    src = _source(runner, s)
    if src is None:
        return None
    props = runner.ctx._props
    chunk = int(props.get("StreamChunkBytes") or DEFAULT_CHUNK_BYTES)
    force = bool(props.get("StreamStages"))
    big = max((_partition_bytes(src[0], src[1], p) for p in range(s.partitions)), default=0)
    if not force and big <= chunk:
        return None
    return dict(kind=src[0], info=src[1], chunk=chunk)


class NotStreamable(Exception):
    """The first chunk's output has no fixed record layout the part writer could encode (the
    vertex then runs unstreamed)."""


def _chunks(plan, p, device, vctx):
    """Yield the DeviceTable of each chunk of partition p of the source."""
    kind, info, chunk = plan["kind"], plan["info"], plan["chunk"]
    if kind == "hostrows":
        h = info["local"].get(p)
        if h is None or h.n == 0:
            return
        per = max(1, chunk // h.stride)
        for a in range(0, h.n, per):
            m = min(per, h.n - a)
            buf = torch.empty((m, h.stride), dtype=torch.uint8, device=device)
            buf.copy_(h.rows[a: a + m], non_blocking=h.pinned)
            yield DeviceTable(m, Shape("rows", key_off=h.key_off, key_len=h.key_len), rows=buf)
        return
    if kind == "hostcols":
        h = info["local"].get(p)
        if h is None or h.n == 0:
            return
        per_row = max(1, h.nbytes // max(h.n, 1))
        yield from h.device_pieces(device, max(1, chunk // per_row))
        return
    if kind == "rows":
        from ..io import reader as RD
        mm, ko, kl = info["prov"].rows_part(info["uri"], p)
        n, w = mm.shape
        per = max(1, chunk // w)
        for a in range(0, n, per):
            m = min(per, n - a)
            # a fresh buffer per chunk: the writer may still be DMA-ing the previous one out
            # (the allocator recycles it after those copies, PartWriter.write records the stream)
            buf = torch.empty((m, w), dtype=torch.uint8, device=device)
            RD.read_rows_to_device(mm.filename, device, int(mm.offset) + a * w, m, w, buf,
                                   stats=vctx.runner.read_stats)
            yield DeviceTable(m, Shape("rows", key_off=ko, key_len=kl), rows=buf)
        return
    if kind == "fixed":
        from ..io import partfile as PF
        from ..io import reader as RD
        from ..ops import codec as CD
        path = PF.read_meta(parse_uri(info["uri"])[1]).part_path(p)
        w = info["width"]
        n = os.path.getsize(path) // w
        per = max(1, chunk // w)
        for a in range(0, n, per):
            m = min(per, n - a)
            raw = RD.read_to_device(path, device, offset=a * w, length=m * w, stats=vctx.runner.read_stats)
            yield CD.decode(raw, info["dtype"])
        return
    from ..io.providers import GenProvider
    lo, hi = GenProvider().bounds(info["uri"], p)
    q = info["q"]
    if kind == "terasort":
        from ..ops import terasort as TSK
        per = max(1, chunk // 100)
        for a in range(lo, hi, per):
            m = min(per, hi - a)
            rows = torch.empty((m, 100), dtype=torch.uint8, device=device)
            TSK.generate(rows, a, int(q.get("seed", 0)))
            yield DeviceTable(m, Shape("rows", key_off=0, key_len=10), rows=rows)
        return
    if kind == "records64":
        from ..models.records_cpu import FIELDS, dim_multiplier
        from ..ops import relational as R
        ncols = int(q.get("cols", 8))
        nk = int(q.get("keys", 1 << 20))
        per = max(1, chunk // (8 * ncols))
        for a in range(lo, hi, per):
            m = min(per, hi - a)
            cols = [torch.empty(m, dtype=torch.int64, device=device) for _ in range(ncols)]
            R.gen_records64(cols, a, nk, int(q.get("seed", 0)), dim_multiplier(nk) if q.get("mode") == "dim" else 0)
            names = FIELDS[:ncols]
            yield DeviceTable.from_columns(dict(zip(names, cols)), Shape("tuple", names))
        return
    if kind == "names":
        from ..models import names as NM
        from ..models.records_cpu import dim_multiplier
        nk = int(q.get("keys", 1 << 20))
        per = max(1, chunk // 32)
        for a in range(lo, hi, per):
            m = min(per, hi - a)
            yield NM.device_table(a, m, nk, int(q.get("seed", 0)), dim_multiplier(nk) if q.get("mode") == "dim" else 0,
                                  device, NM.namelen(q))
        return
    if kind == "range":
        start = int(q.get("start", 0))
        per = max(1, chunk // 8)
        for a in range(lo, hi, per):
            m = min(per, hi - a)
            dt = torch.int32 if start + hi < 2 ** 31 else torch.int64
            yield DeviceTable.from_columns({"v": torch.arange(start + a, start + a + m, dtype=dt, device=device)},
                                           Shape("scalar", ["v"]))
        return
    raise ValueError(kind)


def _encode(t, dtype):
    """(bytes tensor, rows format dict | None) of one output chunk in the part's format."""
    from ..io import binary as B
    from ..ops import codec as CD
    from .gpu_executor import _to_objects
    if isinstance(t, DeviceTable) and t.rows is not None and t.shape.kind == "rows":
        return t.rows[: t.n].contiguous(), dict(stride=t.rows.shape[1], key_off=t.shape.key_off,
                                                key_len=t.shape.key_len)
    if isinstance(t, DeviceTable):
        data = CD.encode(t, dtype)
        if data is None:
            enc = CD.encode_var(t, dtype)
            data = enc[0] if enc is not None else None
        if data is not None:
            return data, None
    raw = B.encode_records(dtype, t if isinstance(t, list) else _to_objects(t))
    return (torch.frombuffer(bytearray(raw), dtype=torch.uint8) if raw else torch.empty(0, dtype=torch.uint8)), None


def run(runner, s, p, version, vctx, plan, cancel=None):
    """Stream partition p of stage s chunk by chunk into a tmp part file -> StreamedPart."""
    from ..io import partfile as PF
    from ..io import writer as WR
    from .grace_stage import StreamedPart
    from .gpu_executor import VertexCancelled
    _, path, _ = parse_uri(s.output["uri"])
    base = PF.default_base(path)
    os.makedirs(os.path.dirname(base) or ".", exist_ok=True)
    tmp = f"{PF.tmp_part_path(base, p, runner.vids[s.id][p], 0, version)}.stream"
    from .grace_stage import _table_dtype
    from .. import types as T
    from ..gpu.stats import BoundsAcc
    n, rows_fmt, chunks = 0, None, 0
    acc = BoundsAcc()
    dtype = None if s.dtype in (None, T.Pickle) else s.dtype    # unknown: the first chunk decides
    with WR.PartWriter(tmp, vctx.device, runner.write_stats) as w:
        for t in _chunks(plan, p, vctx.device, vctx):
            if cancel is not None and cancel.is_set():
                raise VertexCancelled(f"{s.name}[{p}] v{version}")
            data = t
            for op in s.ops[1:-1]:
                data = runner._run_op(op, [data], vctx, s)
            data = runner._run_op(s.ops[-1], [data], vctx, s)
            is_rows = isinstance(data, DeviceTable) and data.rows is not None and data.shape.kind == "rows"
            if dtype is None and not is_rows:
                # the plan does not know the record type: the first chunk's columns decide it
                dtype = _table_dtype(data) if isinstance(data, DeviceTable) else None
                if dtype is None:
                    raise NotStreamable(f"{s.name}: no fixed record layout to stream")
            b, rf = _encode(data, dtype)
            rows_fmt = rows_fmt or rf
            acc.add(data)
            w.write(b)
            n += data.n if isinstance(data, DeviceTable) else len(data)
            chunks += 1
    runner.stream_stats[(s.id, p)] = dict(chunks=chunks, records=n, bytes=w.off)
    return StreamedPart(tmp, n, w.off, dtype, rows=rows_fmt, bounds=acc.result())


def partition_plan(runner, s):
    """``read -> (Select | Where)* -> HashPartition -(cross)-> ToStore(partfile)`` over one source
    partition on one rank: the chunks' ports stream straight into the output's part files (one
    multi-file writer), so the partition never has to fit in HBM.  None when not applicable."""
    if not runner.gpu_ok or runner.world.size != 1 or s.inputs or s.partitions != 1 or len(s.ops) < 2:
        return None
    if s.ops[-1]["op"] != "hash_partition" or any(o["op"] not in STREAM_OPS for o in s.ops[1:-1]):
        return None
    if s.id in runner.skipped or s.id in runner.gang_stages:
        return None
    cons = runner.plan.consumers(s.id)
    if len(cons) != 1:
        return None
    B = runner.plan.stages[cons[0]]
    if [o["op"] for o in B.ops] != ["output"] or not B.is_output or len(B.inputs) != 1 or B.inputs[0].kind != "cross":
        return None
    if parse_uri(B.output["uri"])[0] not in ("partfile", "file") or runner.ctx.OutputDataCompressionScheme.value != 0:
        return None
    src = _source(runner, s)
    if src is None:
        return None
    props = runner.ctx._props
    chunk = int(props.get("StreamChunkBytes") or DEFAULT_CHUNK_BYTES)
    if not props.get("StreamStages") and _partition_bytes(src[0], src[1], 0) <= chunk:
        return None
    return dict(kind=src[0], info=src[1], chunk=chunk, out_stage=B)


def run_partitioned(runner, s, p, version, vctx, plan):
    """Stream partition p of stage s through its HashPartition into the output stage's part
    files -> [StreamedPart per output partition] (the cross edge hands port k to partition k)."""
    from ..io import partfile as PF
    from ..io import writer as WR
    from .grace_stage import StreamedPart, _table_dtype
    from .. import types as T
    B = plan["out_stage"]
    nparts = B.partitions
    _, path, _ = parse_uri(B.output["uri"])
    base = PF.default_base(path)
    os.makedirs(os.path.dirname(base) or ".", exist_ok=True)
    paths = [f"{PF.tmp_part_path(base, k, runner.vids[B.id][k], 0, version)}.stream" for k in range(nparts)]
    dtype = None if B.dtype in (None, T.Pickle) else B.dtype
    from ..gpu.stats import BoundsAcc
    counts, rows_fmt, chunks = [0] * nparts, None, 0
    accs = [BoundsAcc() for _ in range(nparts)]
    w = WR.PartWriter(paths, vctx.device, runner.write_stats)
    try:
        for t in _chunks(plan, p, vctx.device, vctx):
            data = t
            for op in s.ops[1:]:
                data = runner._run_op(op, [data], vctx, s)
            for k in range(nparts):
                piece = data.port(k)
                if piece is None or (hasattr(piece, "n") and piece.n == 0):
                    continue
                is_rows = isinstance(piece, DeviceTable) and piece.rows is not None and piece.shape.kind == "rows"
                if dtype is None and not is_rows:
                    dtype = _table_dtype(piece) if isinstance(piece, DeviceTable) else None
                    if dtype is None:
                        raise NotStreamable(f"{s.name}: no fixed record layout to stream")
                b, rf = _encode(piece, dtype)
                rows_fmt = rows_fmt or rf
                accs[k].add(piece)
                w.write(b, file=k)
                counts[k] += piece.n if isinstance(piece, DeviceTable) else len(piece)
            chunks += 1
        sizes = w.close()
    except BaseException:
        w.abort()
        for f in paths:
            try:
                os.remove(f)
            except OSError:
                pass
        raise
    runner.stream_stats[(s.id, p)] = dict(chunks=chunks, records=sum(counts), bytes=sum(sizes), ports=nparts,
                                          kind="streamed partition to store")
    return [StreamedPart(paths[k], counts[k], sizes[k], dtype, rows=rows_fmt, bounds=accs[k].result())
            for k in range(nparts)]

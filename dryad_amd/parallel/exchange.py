"""Device channels between ranks: DeviceTables moved by RCCL all-to-all-v, column by column.

The reference moves every cross-vertex channel as a file served over HTTP
(``DrOutputGenerator.cpp:216-224``, ``ProcessService/HttpServer.cs:622-660``); a CrossProduct
shuffle is N x M such files (``GraphBuilder.cs:481-504``).  Here a channel between GPUs is a slice
of an HBM table, and one stage's worth of channels is ONE exchange:

  * a manifest as two small tensor collectives (header all-gather: structure digest and column
    dtypes; all-to-all of piece row counts and string-heap bytes) so every rank sizes its receive
    buffers and agrees on column types (partitions whose inferred widths differ, e.g. Int32 vs
    Int64 columns, are promoted);
  * one asynchronous all-to-all-v per column over xGMI, all queued back to back (RCCL ``all_to_all_single``; the send side is a view of
    the producer's port-grouped columns whenever the pieces for consecutive ranks are adjacent,
    which is what the rank-major partition order of ``gpu/ops`` guarantees, so nothing is packed);
  * one more all-to-all-v per string field: the pieces' string bytes compacted in row order
    (``ops/channel.compact_heap``); receivers rebuild offsets as the prefix sum of the lengths.

No record ever becomes a Python object, and no rank receives data it does not consume.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..gpu.table import DeviceTable, Shape
from ..ops import channel as CH
from . import shuffle
from .comm import World


class SchemaMismatch(Exception):
    """Ranks hold structurally different tables: the caller has to use the object transport."""


# ------------------------------------------------------------------------------------------------
def _string_specs(t: DeviceTable) -> list:
    """(offset column, length column, heap key) of every variable-length field."""
    if t.heap is not None:
        return [("off", "len", None)]
    return [(f, f + "#len", f) for f in t.strs]


def _columns(t: DeviceTable) -> dict:
    if t.rows is not None:
        return {"__rows__": t.rows}
    return t.cols


def signature(t: DeviceTable):
    """(structure, dtypes): the structure must match across ranks, dtypes may be promoted."""
    cols = _columns(t)
    sh = t.shape
    struct = (sh.kind, tuple(sh.fields), sh.pytype, sh.key_off, sh.key_len,
              tuple((k, tuple(v.shape[1:])) for k, v in cols.items()), tuple(_string_specs(t)))
    return struct, tuple(str(v.dtype) for v in cols.values())


def _dtype(name: str) -> torch.dtype:
    return getattr(torch, name.split(".")[-1])


def _dense(t: torch.Tensor) -> bool:
    """Row-major with the standard strides in EVERY dim (is_contiguous() accepts any stride on a
    dim of size 1, e.g. a one-row slice of an entries column, which a byte view cannot take)."""
    exp = 1
    for d in range(t.dim() - 1, -1, -1):
        if t.stride(d) != exp:
            return False
        exp *= t.shape[d]
    return True


def _span(ts: list):
    """A view covering tensors that are consecutive contiguous slices of one storage, else None."""
    if not ts:
        return None
    base = ts[0]
    try:
        st = base.untyped_storage()
    except RuntimeError:
        return None
    pos = base.storage_offset()
    end = pos
    for t in ts:
        if t.dtype != base.dtype or not _dense(t) or t.untyped_storage().data_ptr() != st.data_ptr() \
                or t.storage_offset() != end or t.shape[1:] != base.shape[1:]:
            return None
        end += t.numel()
    out = torch.empty(0, dtype=base.dtype, device=base.device)
    tail = tuple(base.shape[1:])
    per = 1
    for d in tail:
        per *= d
    out.set_(st, pos, ((end - pos) // max(per, 1),) + tail)
    return out


def _cat(ts: list, like: torch.Tensor):
    if not ts:
        return like.new_empty((0,) + tuple(like.shape[1:]))
    nonempty = [t for t in ts if t.shape[0] > 0]
    if not nonempty:
        return ts[0]
    if len(nonempty) == 1:
        return nonempty[0]
    sp = _span(nonempty)
    return sp if sp is not None else torch.cat([t.contiguous() for t in nonempty])


def _bytes(t: torch.Tensor) -> torch.Tensor:
    if t.numel() == 0:
        return torch.empty(0, dtype=torch.uint8, device=t.device)
    if not _dense(t):
        t = torch.empty(t.shape, dtype=t.dtype, device=t.device).copy_(t)
    return t.reshape(-1).view(torch.uint8)


class ExchangeStats:
    def __init__(self):
        self.bytes_sent = 0
        self.bytes_received = 0
        self.collectives = 0


# dtype codes of the tensor manifest (index in this list)
_DTYPES = [torch.bool, torch.uint8, torch.int8, torch.int16, torch.int32, torch.int64, torch.float16,
           torch.bfloat16, torch.float32, torch.float64]
_MAXC = 64                     # columns a manifest header carries


def _struct_hash(struct) -> int:
    """A 63-bit digest of a table structure (identical structures on every rank hash alike)."""
    import hashlib
    return int.from_bytes(hashlib.blake2b(repr(struct).encode(), digest_size=8).digest(), "little") >> 1


_BOUNDS_AT = 5 + _MAXC         # header slots of the per-column bounds
_I64_MIN, _I64_MAX = -(1 << 63), (1 << 63) - 1


def _sent_bounds(sends: list, name: str):
    """(lo, hi) over every piece this rank sends of integer column ``name`` when all of them have
    registered bounds ((I64_MAX, I64_MIN) when it sends no rows), else None."""
    from ..gpu import stats as ST
    lo, hi = _I64_MAX, _I64_MIN
    for lst in sends:
        for p in lst:
            if p is None or p.n == 0:
                continue
            c = _columns(p).get(name)
            if c is None or c.dtype in (torch.bool,) or c.is_floating_point() or c.is_complex():
                return None
            b = ST.known(c)
            if b is None:
                return None
            lo, hi = min(lo, b[0]), max(hi, b[1])
    return lo, hi


def _manifest(world: World, sends: list, proto):
    """The exchange's control plane as two small tensor collectives instead of pickled objects:
    an all-gather of each rank's header (has a piece, structure digest, column dtypes, string
    fields, pieces per destination) and an all-to-all of per-destination piece sizes (rows and
    string bytes per piece).  Returns (headers [W][...], pieces[s] = [(rows, [string bytes])] that
    rank s sends here, in order)."""
    W = world.size
    dev = world.device if world.backend == "nccl" else torch.device("cpu")
    sig = signature(proto) if proto is not None else None
    nstr = len(_string_specs(proto)) if proto is not None else 0
    if sig is not None and len(sig[1]) > _MAXC:
        raise SchemaMismatch(f"tables of more than {_MAXC} columns travel as objects")
    # string bytes per piece: every length column summed on the device, one host read for all
    sums = [p.cols[lc][:p.n].sum().to(torch.int64) for lst in sends for p in lst if p.n
            for _, lc, _ in _string_specs(p)]
    vals = iter(torch.stack(sums).tolist() if sums else [])
    per_dest = [[(p.n, [next(vals) if p.n else 0 for _ in range(nstr)]) for p in lst] for lst in sends]
    maxp = max((len(x) for x in per_dest), default=0)
    hdr = torch.zeros(_BOUNDS_AT + 3 * _MAXC, dtype=torch.int64)
    if sig is not None:
        hdr[0], hdr[1], hdr[2], hdr[3] = 1, _struct_hash(sig[0]), len(sig[1]), nstr
        for j, d in enumerate(sig[1]):
            if _dtype(d) not in _DTYPES:
                raise SchemaMismatch(f"column dtype {d} has no manifest code")
            hdr[5 + j] = _DTYPES.index(_dtype(d))
        # the column bounds this rank's pieces carry (gpu/stats.py): known, lo, hi per column
        for j, name in enumerate(_columns(proto)):
            b = _sent_bounds(sends, name)
            if b is not None:
                hdr[_BOUNDS_AT + 3 * j: _BOUNDS_AT + 3 * j + 3] = torch.tensor([1, b[0], b[1]], dtype=torch.int64)
    hdr[4] = maxp
    heads = shuffle.all_gather_tensor(hdr.view(1, -1).to(dev), world).cpu().tolist()
    M = max(h[4] for h in heads)
    S = max(h[3] for h in heads)
    rec = 1 + M * (1 + S)
    out = torch.zeros((W, rec), dtype=torch.int64)
    for r, lst in enumerate(per_dest):
        out[r, 0] = len(lst)
        for i, (n, sb) in enumerate(lst):
            out[r, 1 + i * (1 + S)] = n
            for j, b in enumerate(sb):
                out[r, 2 + i * (1 + S) + j] = b
    got = out.clone()
    if W > 1:
        send_t, recv_t = out.to(dev).view(-1), torch.empty(W * rec, dtype=torch.int64, device=dev)
        dist.all_to_all_single(recv_t, send_t)
        got = recv_t.view(W, rec).cpu()
    g = got.tolist()
    pieces = [[(g[s][1 + i * (1 + S)], g[s][2 + i * (1 + S): 2 + i * (1 + S) + S]) for i in range(g[s][0])]
              for s in range(W)]
    return heads, pieces


def _set_received_bounds(have: list, colspecs, out_cols: dict, offset_cols: set) -> None:
    """A received integer column holds the union of what the senders held: it keeps their bounds
    when every sender knew them (its consumer then skips a min/max pass, gpu/stats.py)."""
    from ..gpu import stats as ST
    for j, (name, _) in enumerate(colspecs):
        col = out_cols.get(name)
        if name in offset_cols or name == "__rows__" or not isinstance(col, torch.Tensor) \
                or col.is_floating_point() or col.dtype == torch.bool or j >= _MAXC:
            continue
        at = _BOUNDS_AT + 3 * j
        if not all(h[at] == 1 for h in have):
            continue
        lo, hi = min(h[at + 1] for h in have), max(h[at + 2] for h in have)
        if lo <= hi:
            ST.set_bounds(col, lo, hi)


def exchange(world: World, sends: list, stats: ExchangeStats | None = None) -> list:
    """``sends[r]``: DeviceTables (pieces) for rank r, in order.  Returns ``recv[s]``: the pieces
    rank s sent to this rank, in its order.  Collective: every rank calls it with W send lists.
    Raises SchemaMismatch (on every rank) when the ranks' tables are structurally different."""
    return exchange_start(world, sends, stats).finish()


def _structure(world: World, have_rank: int, proto):
    """The table structure from rank ``have_rank`` (the first rank holding a piece), for ranks
    that hold none: its repr-free pickle broadcast as one uint8 tensor (length, then bytes) -- no
    object collective."""
    import pickle
    dev = world.device if world.backend == "nccl" else torch.device("cpu")
    me = world.rank
    blob = pickle.dumps(signature(proto)[0]) if me == have_rank else b""
    ln = torch.tensor([len(blob)], dtype=torch.int64, device=dev)
    dist.broadcast(ln, src=have_rank)
    buf = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(dev) if me == have_rank else \
        torch.empty(int(ln.item()), dtype=torch.uint8, device=dev)
    dist.broadcast(buf, src=have_rank)
    return pickle.loads(buf.cpu().numpy().tobytes())     # this framework's own structure tuple


class RecvArena:
    """Receive buffers of consecutive exchanges laid back to back, one region per column: the
    pieces a partition receives over many rounds (a streamed shuffle holding them for one final
    reduce, runtime/stream_shuffle.py) then concatenate as ONE view (DeviceTable._adjacent) instead
    of a copy.  ``nbytes`` is split over the columns by their row widths at the first round; a
    round that no longer fits gets fresh buffers (its pieces are then copied when concatenated)."""

    def __init__(self, nbytes: int, device):
        self.nbytes, self.dev = int(nbytes), device
        self.bufs, self.used, self.rows = None, None, 0

    def take(self, widths: dict, rows: int):
        """{column: uint8 buffer of rows * width bytes} for the next round, or None when the
        arena's column layout differs or it has no room left."""
        if self.bufs is None:
            per = sum(widths.values())
            if per <= 0:
                return None
            self.rows = self.nbytes // per
            self.bufs = {k: torch.empty(self.rows * w, dtype=torch.uint8, device=self.dev) for k, w in widths.items()}
            self.widths, self.used = dict(widths), 0
        if widths != self.widths or self.used + rows > self.rows:
            return None
        out = {k: self.bufs[k][self.used * w: (self.used + rows) * w] for k, w in widths.items()}
        self.used += rows
        return out


class PendingExchange:
    """An exchange whose payload collectives are queued (asynchronous all-to-all-v per column and
    per string heap) but not yet waited for; ``finish()`` makes the caller's stream wait and
    returns the received pieces.  The send buffers stay referenced until then."""

    def __init__(self, W, recv_pieces, big_args, handles, strs, keep):
        self.W, self.recv_pieces, self.big_args = W, recv_pieces, big_args
        self.handles, self.strs, self.keep = handles, strs, keep

    def finish(self) -> list:
        if self.big_args is None:
            return [[] for _ in range(self.W)]
        for h in self.handles:
            shuffle.wait(h)
        total_r, shape, out_cols, heaps, have, colspecs, offset_cols = self.big_args
        for oc, lc, hk, recv in self.strs:         # offsets rebuilt from the received lengths
            ln = out_cols[lc].to(torch.int64)
            out_cols[oc] = (torch.cumsum(ln, 0) - ln).to(out_cols[oc])
            heaps[hk] = recv
        _set_received_bounds(have, colspecs, out_cols, offset_cols)
        if "__rows__" in out_cols:
            big = DeviceTable(total_r, shape, rows=out_cols["__rows__"])
        else:
            big = DeviceTable(total_r, shape, out_cols, heap=heaps.get(None),
                              strs={k: v for k, v in heaps.items() if k is not None})
        res, a = [], 0
        for s in range(self.W):
            lst = []
            for n, _ in self.recv_pieces[s]:
                lst.append(big.slice(a, a + n))
                a += n
            res.append(lst)
        self.keep = None
        return res


def exchange_start(world: World, sends: list, stats: ExchangeStats | None = None,
                   arena: RecvArena | None = None) -> PendingExchange:
    """Queue an exchange (see ``exchange``).  The manifest is two tensor collectives
    (``_manifest``); the payload columns and string heaps are queued as asynchronous all-to-all-v
    collectives back to back (RCCL runs them in order on its stream while the host prepares the
    next, and while the caller computes); a partition's received pieces are adjacent slices of one
    buffer per column (DeviceTable.concat takes them as one view)."""
    W, me = world.size, world.rank
    assert len(sends) == W
    proto = next((p for lst in sends for p in lst if p is not None), None)
    heads, recv_pieces = _manifest(world, sends, proto)
    have = [h for h in heads if h[0]]
    if not have:                      # nobody holds a piece
        return PendingExchange(W, recv_pieces, None, [], [], None)
    if len({h[1] for h in have}) != 1 or len({h[2] for h in have}) != 1:
        raise SchemaMismatch("ranks hold different table structures")
    if len(have) < W:
        # a rank without source pieces learns the structure from the first rank that has one (rare:
        # fewer source partitions than ranks); every rank sees the same headers, so all take this branch
        struct = _structure(world, next(r for r, h in enumerate(heads) if h[0]), proto)
    else:
        struct = signature(proto)[0]
    kind, fields, pytype, key_off, key_len, colspecs, strspecs = struct
    dtypes = []
    for j in range(len(colspecs)):
        dt = _DTYPES[have[0][5 + j]]
        for h in have[1:]:
            dt = torch.promote_types(dt, _DTYPES[h[5 + j]])
        dtypes.append(dt)
    shape = Shape(kind, list(fields), pytype, key_off, key_len)
    dev = world.device if world.device.type == "cuda" else (proto.device if proto is not None else torch.device("cpu"))
    recv_rows = [sum(n for n, _ in recv_pieces[s]) for s in range(W)]
    send_rows = [sum(p.n for p in sends[r]) for r in range(W)]
    total_r = sum(recv_rows)
    out_cols = {name: None for name, _ in colspecs}
    offset_cols = {oc for oc, _, _ in strspecs}        # rebuilt from the lengths on arrival
    handles, keep = [], []
    slots = None
    if arena is not None and not strspecs:
        widths = {}
        for (name, tail), dt in zip(colspecs, dtypes):
            per = torch.empty((0,) + tuple(tail), dtype=dt).element_size()
            for d in tail:
                per *= d
            widths[name] = per
        slots = arena.take(widths, total_r)
    for (name, tail), dt in zip(colspecs, dtypes):
        if name in offset_cols:
            out_cols[name] = dt
            continue
        per = torch.empty((0,) + tuple(tail), dtype=dt).element_size()
        for d in tail:
            per *= d
        pieces = [_columns(p)[name][:p.n] for lst in sends for p in lst]
        pieces = [x if x.dtype == dt else x.to(dt) for x in pieces]
        like = torch.empty((0,) + tuple(tail), dtype=dt, device=dev)
        send = _bytes(_cat(pieces, like)) if pieces else torch.empty(0, dtype=torch.uint8, device=dev)
        recv = slots[name] if slots is not None else torch.empty(total_r * per, dtype=torch.uint8, device=dev)
        handles.append(shuffle.alltoallv_bytes_async(send, [c * per for c in send_rows], recv,
                                                     [c * per for c in recv_rows], world))
        keep.append(send)
        out_cols[name] = recv.view(dt).view((total_r,) + tuple(tail))
        if stats is not None:
            stats.bytes_sent += sum(send_rows) * per
            stats.bytes_received += total_r * per
            stats.collectives += 1
    heaps, strs = {}, []
    for j, (oc, lc, hk) in enumerate(strspecs):
        parts, send_b = [], []
        for lst in sends:
            nb = 0
            for p in lst:
                if p.n == 0:
                    continue
                heap = p.heap if hk is None else p.strs[hk]
                h, _ = CH.compact_heap(heap, p.cols[oc][:p.n], p.cols[lc][:p.n])
                parts.append(h)
                nb += h.numel()
            send_b.append(nb)
        recv_b = [sum(sb[j] for _, sb in recv_pieces[s]) for s in range(W)]
        send = torch.cat(parts) if len(parts) > 1 else (parts[0] if parts else torch.empty(0, dtype=torch.uint8,
                                                                                                device=dev))
        recv = torch.empty(sum(recv_b), dtype=torch.uint8, device=dev)
        handles.append(shuffle.alltoallv_bytes_async(send, send_b, recv, recv_b, world))
        keep.append(send)
        strs.append((oc, lc, hk, recv))
        if stats is not None:
            stats.bytes_sent += sum(send_b)
            stats.bytes_received += recv.numel()
            stats.collectives += 1
    return PendingExchange(W, recv_pieces, (total_r, shape, out_cols, heaps, have, colspecs, offset_cols),
                           handles, strs, keep)

"""Shuffle engine: the Dryad CrossProduct channel pattern as RCCL collectives over xGMI.

Reference mapping:
  * R1 HashPartition/RangePartition -> Merge (``GraphBuilder.ConnectCrossProduct``, N x M files
    served over HTTP) becomes a size exchange (all-to-all of int64 counts) followed by one
    all-to-all-v of the payload.  On a fully connected 8-GPU xGMI node every GPU drives its 7
    links concurrently, so the exchange is pairwise (alltoallv), never a ring.
  * R2 full merge to one partition -> gather to the root.
  * R3 Tee broadcast -> broadcast / all-gather.
  * R4 aggregation trees -> all-reduce (dense) or all-to-all + local combine (sparse keys).
  * R5 sampler gather -> all-gather of the samples.

Large exchanges are issued in chunks (``CHUNK_BYTES``, 4 GiB per peer per round) so that RCCL's internal staging and the int32 limits of some code paths are never hit and
so a later version can overlap the next chunk's pack kernel with the current transfer.
"""
from __future__ import annotations


import torch
import torch.distributed as dist

from .comm import World, get_world

CHUNK_BYTES = 4 << 30         # per (source, destination) pair and round (tests shrink it)


def exchange_counts(send_counts: torch.Tensor, world: World | None = None) -> torch.Tensor:
    """All-to-all of per-destination counts (int64 [world]).  Returns the receive counts."""
    w = world or get_world()
    if not w.collective:
        return send_counts.clone()
    dev = w.device if w.backend == "nccl" else torch.device("cpu")
    s = send_counts.to(dev, torch.int64).contiguous()
    r = torch.empty_like(s)
    dist.all_to_all_single(r, s)
    return r.to(send_counts.device)


def _native(w: World, *tensors) -> bool:
    """The tensors live where the backend moves data itself: HBM under RCCL, host memory under
    gloo.  These transfers take the collective branches (async handles, split sizes, chunked P2P
    rounds); a gloo CPU run exercises exactly the code an RCCL run executes."""
    want_cuda = w.backend == "nccl"
    return all(t.is_cuda == want_cuda for t in tensors)


def alltoallv_bytes(send: torch.Tensor, send_counts: list[int], recv: torch.Tensor, recv_counts: list[int],
                    world: World | None = None):
    """All-to-all-v over flat uint8 views: ``send`` is grouped by destination with
    ``send_counts[d]`` bytes for rank d; ``recv`` receives ``recv_counts[s]`` bytes from rank s,
    in source-rank order."""
    w = world or get_world()
    assert send.dtype == torch.uint8 and recv.dtype == torch.uint8
    if not w.collective:
        n = send_counts[0]
        recv[:n].copy_(send[:n])
        return recv
    assert len(send_counts) == w.size and len(recv_counts) == w.size
    total_s, total_r = sum(send_counts), sum(recv_counts)
    assert send.numel() >= total_s and recv.numel() >= total_r
    if not _native(w, send, recv):
        # gloo transport for device buffers (tests / shared-GPU ranks): stage through host memory
        s_cpu = send[:total_s].cpu()
        r_cpu = torch.empty(total_r, dtype=torch.uint8)
        dist.all_to_all_single(r_cpu, s_cpu, output_split_sizes=list(recv_counts),
                               input_split_sizes=list(send_counts))
        recv[:total_r].copy_(r_cpu)
        return recv
    maxpair = max(max(send_counts), max(recv_counts))
    if maxpair <= CHUNK_BYTES:
        dist.all_to_all_single(recv[:total_r], send[:total_s], output_split_sizes=list(recv_counts),
                               input_split_sizes=list(send_counts))
        return recv
    # chunked rounds: every round moves up to CHUNK_BYTES from each source to each destination
    soff = [0] * w.size
    roff = [0] * w.size
    acc = 0
    for d in range(w.size):
        soff[d] = acc
        acc += send_counts[d]
    acc = 0
    for s_ in range(w.size):
        roff[s_] = acc
        acc += recv_counts[s_]
    done_s = [0] * w.size
    done_r = [0] * w.size
    while any(done_s[d] < send_counts[d] for d in range(w.size)) or any(
            done_r[s_] < recv_counts[s_] for s_ in range(w.size)):
        ops = []
        for peer in range(w.size):
            ns = min(CHUNK_BYTES, send_counts[peer] - done_s[peer])
            nr = min(CHUNK_BYTES, recv_counts[peer] - done_r[peer])
            if peer == w.rank:
                if ns > 0:
                    recv[roff[peer] + done_r[peer]: roff[peer] + done_r[peer] + nr].copy_(
                        send[soff[peer] + done_s[peer]: soff[peer] + done_s[peer] + ns])
            else:
                if ns > 0:
                    ops.append(dist.P2POp(dist.isend, send[soff[peer] + done_s[peer]: soff[peer] + done_s[peer] + ns],
                                          peer))
                if nr > 0:
                    ops.append(dist.P2POp(dist.irecv, recv[roff[peer] + done_r[peer]: roff[peer] + done_r[peer] + nr],
                                          peer))
            done_s[peer] += max(ns, 0)
            done_r[peer] += max(nr, 0)
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()
    return recv


def alltoallv_bytes_async(send: torch.Tensor, send_counts: list[int], recv: torch.Tensor, recv_counts: list[int],
                          world: World | None = None):
    """``alltoallv_bytes`` that does not wait: over RCCL the collective is queued on the
    communicator's stream and the caller's stream keeps running; ``wait(handle)`` later makes the
    caller's stream wait for it (the pipelined range shuffle sorts sub-range b while round b+1 is
    on the wire).  Other transports (gloo staging through the host, rounds chunked past
    CHUNK_BYTES per peer) complete before returning and give ``None``."""
    w = world or get_world()
    if (w.collective and _native(w, send, recv)
            and max(max(send_counts), max(recv_counts)) <= CHUNK_BYTES):
        ts, tr = sum(send_counts), sum(recv_counts)
        return dist.all_to_all_single(recv[:tr], send[:ts], output_split_sizes=list(recv_counts),
                                      input_split_sizes=list(send_counts), async_op=True)
    alltoallv_bytes(send, send_counts, recv, recv_counts, w)
    return None


def wait(handle) -> None:
    """Make the current stream wait for an ``alltoallv_bytes_async`` handle."""
    if handle is not None:
        handle.wait()


def gang_status(ok: bool, value: int = 0, world: World | None = None) -> list[tuple[bool, int]]:
    """Every rank's (ok, value) from one small all-gather: the agreement a gang stage reaches
    before it enters a payload collective (ops/recordsort: a rank whose pre-exchange work failed,
    or whose key range overflows its receive buffer, says so here and every rank stops alike)."""
    w = world or get_world()
    if not w.collective:
        return [(bool(ok), int(value))]
    dev = w.device if w.backend == "nccl" else torch.device("cpu")
    t = torch.tensor([[1 if ok else 0, int(value)]], dtype=torch.int64, device=dev)
    return [(bool(a), int(b)) for a, b in all_gather_tensor(t, w).tolist()]


def digest(obj) -> int:
    """A 63-bit digest of a plain-data value (its repr): what ranks compare in a planning vote
    instead of pickling the value to every peer."""
    import hashlib
    return int.from_bytes(hashlib.blake2b(repr(obj).encode(), digest_size=8).digest(), "little") >> 1


def gather_ints(values: list, world: World | None = None) -> list:
    """Every rank's list of int64 ``values`` (same length everywhere) from one small tensor
    all-gather: [[rank 0's values], [rank 1's], ...]."""
    w = world or get_world()
    if not w.collective:
        return [list(values)]
    dev = w.device if w.backend == "nccl" else torch.device("cpu")
    t = torch.tensor([list(values)], dtype=torch.int64, device=dev)
    return all_gather_tensor(t, w).tolist()


def vote(ok: bool, key=None, world: World | None = None, values: tuple = ()) -> tuple[bool, list]:
    """A planning vote as one tensor all-gather: (every rank ok and every rank's ``key`` equal,
    every rank's ``values``).  Replaces pickled all_gather_object votes on the per-job path."""
    got = gather_ints([1 if ok else 0, digest(key)] + [int(v) for v in values], world)
    agree = all(g[0] for g in got) and len({g[1] for g in got}) == 1
    return agree, [g[2:] for g in got]


def all_gather_tensor(t: torch.Tensor, world: World | None = None) -> torch.Tensor:
    """All-gather equally shaped tensors along dim 0 (R5: sampler gather, R3 broadcast of small data)."""
    w = world or get_world()
    if not w.collective:
        return t.clone()
    dev_ok = (w.backend == "nccl") == t.is_cuda
    src = t if dev_ok else (t.to(w.device) if w.backend == "nccl" else t.cpu())
    out = torch.empty((w.size * src.shape[0],) + tuple(src.shape[1:]), dtype=src.dtype, device=src.device)
    dist.all_gather_into_tensor(out, src.contiguous())
    return out.to(t.device)


def all_gather_varlen(t: torch.Tensor, world: World | None = None) -> torch.Tensor:
    """All-gather tensors whose dim 0 differs per rank."""
    w = world or get_world()
    if not w.collective:
        return t.clone()
    n = torch.tensor([t.shape[0]], dtype=torch.int64, device=t.device)
    ns = all_gather_tensor(n, w).tolist()
    m = max(ns)
    pad = torch.zeros((m,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    pad[: t.shape[0]] = t
    g = all_gather_tensor(pad, w)
    parts = [g[i * m: i * m + ns[i]] for i in range(w.size)]
    return torch.cat(parts, 0)


def gather_json(obj, world: World | None = None) -> list:
    """Every rank's JSON-serialisable ``obj`` (per-rank control data: part-file paths, report
    records, error strings), as UTF-8 JSON bytes in one variable-length tensor all-gather.  Peers'
    data is parsed, never unpickled (dict keys come back as strings, tuples as lists)."""
    import json
    w = world or get_world()
    if not w.collective:
        return [json.loads(json.dumps(obj))]
    raw = json.dumps(obj).encode()
    t = torch.frombuffer(bytearray(raw), dtype=torch.uint8) if raw else torch.zeros(0, dtype=torch.uint8)
    n = torch.tensor([t.numel()], dtype=torch.int64)
    ns = [int(x) for x in all_gather_tensor(n, w).view(-1).tolist()]
    pad = torch.zeros(max(ns), dtype=torch.uint8)
    pad[: t.numel()] = t
    g = all_gather_tensor(pad, w).view(w.size, -1).cpu()
    return [json.loads(bytes(g[r, : ns[r]].numpy()).decode()) for r in range(w.size)]


def all_reduce_(t: torch.Tensor, op: str = "sum", world: World | None = None) -> torch.Tensor:
    w = world or get_world()
    if not w.collective:
        return t
    rop = {"sum": dist.ReduceOp.SUM, "min": dist.ReduceOp.MIN, "max": dist.ReduceOp.MAX}[op]
    if (w.backend == "nccl") != t.is_cuda:
        tmp = t.to(w.device) if w.backend == "nccl" else t.cpu()
        dist.all_reduce(tmp, op=rop)
        t.copy_(tmp)
    else:
        dist.all_reduce(t, op=rop)
    return t


def broadcast_(t: torch.Tensor, src: int = 0, world: World | None = None) -> torch.Tensor:
    w = world or get_world()
    if not w.collective:
        return t
    if (w.backend == "nccl") != t.is_cuda:
        tmp = t.to(w.device) if w.backend == "nccl" else t.cpu()
        dist.broadcast(tmp, src=src)
        t.copy_(tmp)
    else:
        dist.broadcast(t, src=src)
    return t

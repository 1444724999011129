"""parallel/exchange.py on N gloo ranks (CPU or one shared GPU): random DeviceTables of every layout
(scalar, tuple with strings and vectors, text, fixed-width rows, partial-aggregate style) are
hash-partitioned with rank-major ports, exchanged, and checked against what every rank should
receive (recomputed from the deterministic generators of all ranks)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from dryad_amd.gpu.table import DeviceTable, Shape  # noqa: E402
from dryad_amd.parallel import exchange as EXC  # noqa: E402
from dryad_amd.parallel.comm import init_world  # noqa: E402


def make_table(kind, rank, dev, n):
    g = torch.Generator().manual_seed(1000 * rank + n)
    if kind == "scalar":
        dt = torch.int32 if rank % 2 else torch.int64       # promoted across ranks
        return DeviceTable.from_columns({"v": torch.randint(-1000, 1000, (n,), generator=g).to(dt).to(dev)},
                                        Shape("scalar", ["v"]))
    if kind == "tuple_str_vec":
        words = [("w%d" % int(x)) * (int(x) % 4) for x in torch.randint(0, 50, (n,), generator=g)]
        enc = [w.encode() for w in words]
        ln = torch.tensor([len(e) for e in enc], dtype=torch.int64)
        off = torch.cumsum(ln, 0) - ln
        heap = torch.frombuffer(bytearray(b"".join(enc) or b"\0"), dtype=torch.uint8)[: int(ln.sum())].clone()
        cols = {"Item1": torch.randint(0, 10**9, (n,), generator=g).to(dev), "Item2": off.to(dev),
                "Item2#len": ln.to(dev), "Item3": torch.randn((n, 6), generator=g).to(dev),
                "Item4": (torch.randint(0, 2, (n,), generator=g) == 1).to(dev)}
        return DeviceTable(n, Shape("tuple", ["Item1", "Item2", "Item3", "Item4"]), cols, strs={"Item2": heap.to(dev)})
    if kind == "text":
        lines = ["line %d of rank %d" % (i, rank) * (i % 3) for i in range(n)]
        enc = [x.encode() for x in lines]
        ln = torch.tensor([len(e) for e in enc], dtype=torch.int64)
        off = torch.cumsum(ln, 0) - ln
        heap = torch.frombuffer(bytearray(b"".join(enc) or b"\0"), dtype=torch.uint8)[: int(ln.sum())].clone()
        return DeviceTable(n, Shape("text", ["off", "len"], str), {"off": off.to(dev), "len": ln.to(dev)},
                           heap=heap.to(dev))
    if kind == "rows":
        return DeviceTable.from_rows(torch.randint(0, 255, (n, 20), generator=g, dtype=torch.uint8).to(dev), 0, 10)
    raise ValueError(kind)


def dest_of(t, W, nports):
    """Destination port of every row: a hash of its first column (deterministic)."""
    if t.rows is not None:
        key = t.rows[:, 0].to(torch.int64) * 131 + t.rows[:, 1].to(torch.int64)
    else:
        key = next(iter(t.cols.values()))
        key = key.to(torch.int64) if key.dim() == 1 else key[:, 0].to(torch.int64)
    return (key * 2654435761 % 1000003) % nports


def partitioned(t, W, nports, dev):
    from dryad_amd.gpu import ops as G
    e = torch.zeros((t.n, 2), dtype=torch.int64, device=t.device)
    e[:, 1] = dest_of(t, W, nports)
    e[:, 0] = torch.arange(t.n, device=t.device)
    if t.device.type == "cuda":
        return G.partition_by_entries(t, e, nports, W)
    from dryad_amd.ops import channel as CH
    order, lut = G._port_order(nports, W)
    cols = [t.rows] if t.rows is not None else list(t.cols.values())
    outs, cnt = CH.scatter_columns(e, t.n, cols, torch.tensor(lut, dtype=torch.uint8) if lut else None)
    offs = [0]
    for c in cnt[:nports].tolist():
        offs.append(offs[-1] + c)
    from dryad_amd.gpu.table import Ported
    nt = DeviceTable(t.n, t.shape, rows=outs[0]) if t.rows is not None else \
        DeviceTable(t.n, t.shape, dict(zip(t.cols.keys(), outs)), heap=t.heap, strs=t.strs)
    return Ported(nt, offs, order)


def main():
    w = init_world(device=os.environ.get("SPMD_DEVICE", "cpu"))
    W, me = w.size, w.rank
    dev = w.device
    bad = []
    for kind in ("scalar", "tuple_str_vec", "text", "rows"):
        for nports in (W, 2 * W + 1):
            sizes = [(r * 7919 + 13 * nports) % 2000 + (0 if r == 1 else 1) for r in range(W)]
            if kind == "rows":
                sizes[W - 1] = 0                      # a rank with nothing to send
            pt = partitioned(make_table(kind, me, dev, sizes[me]), W, nports, dev)
            sends = [[pt.port(p) for p in range(nports) if p % W == r] for r in range(W)]
            got = EXC.exchange(w, sends)
            for s_ in range(W):
                src = partitioned(make_table(kind, s_, dev, sizes[s_]), W, nports, dev)
                exp = [src.port(p) for p in range(nports) if p % W == me]
                if len(got[s_]) != len(exp):
                    bad.append((kind, nports, s_, "pieces"))
                    continue
                for a, b in zip(got[s_], exp):
                    if a.to_objects() != b.to_objects():
                        bad.append((kind, nports, s_))
            merged = DeviceTable.concat([x for lst in got for x in lst])
            if merged is not None and merged.n != sum(x.n for lst in got for x in lst):
                bad.append((kind, nports, "concat"))
    # a rank holding no piece at all (fewer source partitions than ranks): it learns the table
    # structure from the first rank that has one (a tensor broadcast, no object collective)
    if W > 1:
        t = make_table("tuple_str_vec", me, dev, 50 + me)
        sends = [[] for _ in range(W)] if me == 0 else [[t.slice(0, 25 + me)] if r == 0 else [t.slice(25 + me, t.n)]
                                                         for r in range(W)]
        got = EXC.exchange(w, sends)
        for s_ in range(W):
            want = 0 if s_ == 0 else 1
            if len(got[s_]) != want:
                bad.append(("no-piece", s_, len(got[s_])))
            elif want:
                src = make_table("tuple_str_vec", s_, dev, 50 + s_)
                exp = src.slice(0, 25 + s_) if me == 0 else src.slice(25 + s_, src.n)
                if got[s_][0].to_objects() != exp.to_objects():
                    bad.append(("no-piece", s_, "data"))
    # strided entry columns (views into one [n, 2] tensor, one-row pieces): the merge / broadcast
    # edges of the sampler send such tables unpartitioned
    def ent_table(r, n):
        g = torch.Generator().manual_seed(77 + r)
        e = torch.randint(-2**62, 2**62, (n, 2), generator=g).to(dev)
        return DeviceTable.from_columns({"lo": e[:, 0], "hi": e[:, 1]}, Shape("tuple", ["lo", "hi"]))
    for n in (1, 3):
        t = ent_table(me, n)
        got = EXC.exchange(w, [[t.slice(0, 1), t.slice(1, n)] for _ in range(W)])
        for s_ in range(W):
            e = ent_table(s_, n)
            if [x.to_objects() for x in got[s_]] != [e.slice(0, 1).to_objects(), e.slice(1, n).to_objects()]:
                bad.append(("strided", n, s_))
    # column bounds travel with the pieces (gpu/stats.py): the receiver's concatenation knows the
    # union of the senders' registered bounds; one sender without bounds leaves it unmeasured
    from dryad_amd.gpu import stats as ST
    for unknown_rank in (None, W - 1):
        n = 0 if me == 1 else 50 + me
        col = torch.arange(n, dtype=torch.int64, device=dev) + 100 * me
        if me != unknown_rank:
            ST.set_bounds(col, 100 * me - 5, 100 * me + 60)
        t = DeviceTable.from_columns({"v": col}, Shape("scalar", ["v"]))
        per = (n + W - 1) // W
        got = EXC.exchange(w, [[t.slice(min(r * per, n), min((r + 1) * per, n))] for r in range(W)])
        merged = DeviceTable.concat([x for lst in got for x in lst])
        senders = [r for r in range(W) if r != 1]
        want = None if unknown_rank is not None and unknown_rank != 1 else \
            (min(100 * r - 5 for r in senders), max(100 * r + 60 for r in senders))
        if ST.known(merged.cols["v"]) != want:
            bad.append(("bounds", unknown_rank, ST.known(merged.cols["v"]), want))
    # per-rank control records as JSON over a tensor all-gather (no pickles), uneven sizes
    from dryad_amd.parallel import shuffle as SHF
    got = SHF.gather_json({"rank": me, "paths": [f"/tmp/p{me}.{j}" for j in range(me + 1)], "t": 0.5 * me,
                           "err": None if me else "é boom"}, w)
    if [g["rank"] for g in got] != list(range(W)) or got[W - 1]["paths"][-1] != f"/tmp/p{W - 1}.{W - 1}" \
            or got[0]["err"] != "é boom" or got[1]["t"] != 0.5:
        bad.append(("gather_json", got))
    w.barrier()
    assert not bad, (me, bad[:5])
    if me == 0:
        print("EXCHANGE_OK", W, flush=True)


if __name__ == "__main__":
    main()
    # tear the process group down before the interpreter exits: gloo's threads torn down during
    # finalisation abort the process now and then ("terminate called without an active exception")
    from dryad_amd.parallel.comm import shutdown
    shutdown()

"""Streamed shuffle: a multi-partition GroupBy / Distinct whose partial side and final side run as
one pipelined gang stage with bounded channels (SURVEY C-1, §2.4 CrossProduct).

The planner emits a decomposable GroupBy (or a Distinct) over P partitions as two stages:

    A: read -> (Select | Where)* -> group_partial | distinct -> hash_partition     (no inputs)
    B: group_final | distinct -> ...                                               (cross from A)

Run stage by stage, A's whole partition of partial rows is hash-partitioned, exchanged in one
all-to-all-v per column, and B's partition receives every source's partials at once: the final
GroupBy's input must fit HBM.  The reference never holds it: a vertex consumes its input channels
as streams (RChannelReader, DryadVertex/VertexHost/system/channel/include/channelinterface.h:212;
DryadLinqVertexReader.cs:41-257) and its partial accumulation folds records as they arrive
(ParallelHashGroupByPartialAccumulate, LinqToDryad/DryadLinqVertex.cs:5718).

Here the pair runs as rounds.  Round r: each rank reads its next source chunk
(runtime/streaming._chunks: generator ranges, stored rows, fixed-width parts, host:// tables),
runs A's record-wise operators and partial aggregation on it, hash-partitions the partial rows and
queues them as one asynchronous exchange (parallel/exchange.exchange_start: all-to-all-v per column
and string heap); then it waits for round r-1's pieces and folds them into the running state of
each of its B partitions (runtime/stream_agg.StreamAggregator.add_partial: the directly addressed
dense state of an integer key, or hash buckets spilled to pinned host memory past
``HbmBudgetBytes``).  Round r's transfer overlaps round r+1's partial aggregation and round r-1's
fold.  After the last round each B partition's state is reduced bucket by bucket and streamed to
its output store (runtime/sinks.py) or concatenated for the rest of B's program.

The same rounds serve a plain repartition written to a store,

    A: read -> (Select | Where)* -> hash_partition        B: (Select | Where)* -> output

B's record-wise operators run on each received round and the result goes straight to its
partfile:// / host:// sink (runtime/sinks.py): no stage holds a whole partition.

Chosen when ``StreamShuffle=True`` (context property; False forbids it), or when a source partition
exceeds the HBM budget (the pair could not run stage by stage).  Every rank votes alike.  A round
whose fold fails on one rank (a sink error, out of memory) is agreed at the next round's status
collective, so every rank stops together.
"""
from __future__ import annotations

import time


from ..gpu.table import DeviceTable, Ported
from ..gpu.trace import NotTraceable
from ..parallel import exchange as EXC
from ..parallel import shuffle
from ..utils.log import get_logger
from . import stream_agg as SA
from . import streaming as ST

log = get_logger("stream_shuffle")

PARTIAL_OPS = {"group_partial", "distinct"}
FINAL_OPS = {"group_final", "distinct"}


def _repartition(plan, b):
    """The streamed repartition idiom (A: read -> (Select | Where)* -> hash_partition, B: (Select |
    Where)* -> output), its descriptor or None."""
    st = plan.stages
    if len(b.inputs) != 1 or b.inputs[0].kind != "cross" or not b.ops or b.ops[-1]["op"] != "output":
        return None
    if any(o["op"] not in SA.PRE_OPS for o in b.ops[:-1]):
        return None
    a = st[b.inputs[0].src]
    ops = [o["op"] for o in a.ops]
    if a.inputs or len(ops) < 2 or ops[0] != "read" or ops[-1] != "hash_partition":
        return None
    if any(o not in SA.PRE_OPS for o in ops[1:-1]) or a.is_output or plan.consumers(a.id) != [b.id]:
        return None
    if a.partitions != b.partitions or a.ops[-1].get("count", a.partitions) != b.partitions:
        return None
    return dict(a=a.id, b=b.id, stages=[a.id], mode="repartition")


def find(plan) -> dict:
    """{B stage id: descriptor} for every (A, B) pair of the idioms in the module docstring."""
    out = {}
    st = plan.stages
    for b in st:
        rp = _repartition(plan, b)
        if rp is not None:
            out[b.id] = rp
            continue
        if len(b.inputs) != 1 or b.inputs[0].kind != "cross" or not b.ops or b.ops[0]["op"] not in FINAL_OPS:
            continue
        a = st[b.inputs[0].src]
        ops = [o["op"] for o in a.ops]
        if a.inputs or len(ops) < 3 or ops[0] != "read" or ops[-1] != "hash_partition" or ops[-2] not in PARTIAL_OPS:
            continue
        if any(o not in SA.PRE_OPS for o in ops[1:-2]) or a.is_output or plan.consumers(a.id) != [b.id]:
            continue
        if a.partitions != b.partitions or a.ops[-1].get("count", a.partitions) != b.partitions:
            continue
        pa, fb = a.ops[-2], b.ops[0]
        if (pa["op"] == "distinct") != (fb["op"] == "distinct"):
            continue
        if pa.get("comparer") is not None or fb.get("comparer") is not None:
            continue
        if pa["op"] == "group_partial" and (pa.get("decomp") is None or pa.get("elem") is not None):
            continue
        out[b.id] = dict(a=a.id, b=b.id, stages=[a.id])
    return out


def plan_local(desc, runner):
    """This rank's source plan of stage A (kind, info, chunk bytes, ...) or None."""
    if not runner.gpu_ok:
        return None
    a = runner.plan.stages[desc["a"]]
    src = ST._source(runner, a)
    if src is None:
        return None
    budget = SA._budget(runner)
    me = runner.world.rank
    mine = [p for p in range(a.partitions) if runner.owner(p, a.id) == me]
    if desc.get("mode") == "repartition":
        from . import sinks
        b = runner.plan.stages[desc["b"]]
        owned_b = [p for p in range(b.partitions) if runner.owner(p, b.id) == me]
        if sinks.PartfileSink.applicable(runner, b):
            if len(owned_b) > 1:          # one part writer per process at a time (io/writer.py)
                return None
        elif not sinks.HostSink.applicable(runner, b):
            return None
    big = max((ST._partition_bytes(src[0], src[1], p) for p in mine), default=0)
    props = runner.ctx._props
    chunk = int(props.get("StreamChunkBytes") or ST.DEFAULT_CHUNK_BYTES)
    chunk = max(1 << 20, min(chunk, budget // 8))
    return dict(kind=src[0], info=src[1], chunk=chunk, budget=budget, source_bytes=big)


def vote(desc, runner):
    """Collective (one tensor all-gather): the pair runs streamed iff every rank can and it is
    forced (StreamShuffle=True) or some rank's source partition exceeds its HBM budget."""
    force = runner.ctx._props.get("StreamShuffle")
    lay = None if force is False else plan_local(desc, runner)
    agree, vals = shuffle.vote(lay is not None, None, runner.world,
                               values=(0 if lay is None else int(lay["source_bytes"] > lay["budget"]),))
    if not agree:
        return None
    if force is not True and not any(v[0] for v in vals):
        return None
    return lay


def run(desc, runner, lay) -> dict:
    """Execute the pair on this rank -> {local partition of B: its output value}."""
    from .gpu_executor import GpuVertexContext
    w, dev = runner.world, runner.dev
    W, me = w.size, w.rank
    A, B = runner.plan.stages[desc["a"]], runner.plan.stages[desc["b"]]
    parts_a = [p for p in range(A.partitions) if runner.owner(p, A.id) == me]
    owned = {r: [p for p in range(B.partitions) if runner.owner(p, B.id) == r] for r in range(W)}
    parts_b = owned[me]
    vctx_a = {p: GpuVertexContext(p, A.partitions, runner.vids[A.id][p], 0, A, dev, w, runner) for p in parts_a}
    vctx_b = {p: GpuVertexContext(p, B.partitions, runner.vids[B.id][p], 0, B, dev, w, runner) for p in parts_b}
    rep_mode = desc.get("mode") == "repartition"
    if rep_mode:
        splan = dict(lay, pre=A.ops[1:-1], agg=None, rest=A.ops[-1:])
    else:
        splan = dict(lay, pre=A.ops[1:-2], agg=A.ops[-2], rest=A.ops[-1:])
    # received partials held up to a quarter of the budget (their concatenation doubles it) and
    # reduced once (StreamAggregator.hold_budget)
    bplan = dict(agg=B.ops[0], pre=[], rest=B.ops[1:], budget=lay["budget"], source_bytes=lay["source_bytes"],
                 hold_bytes=lay["budget"] // (4 * max(1, len(parts_b))),
                 chunk=lay["chunk"])
    aggs = {} if rep_mode else {p: SA.StreamAggregator(runner, B, vctx_b[p], dict(bplan)) for p in parts_b}
    # one final partition on this rank: its rounds are received back to back into an arena of the
    # hold budget, so the held partials concatenate as one view for the final reduce
    arena = EXC.RecvArena(bplan["hold_bytes"], dev) if not rep_mode and len(parts_b) == 1 else None
    from . import sinks as SK
    outs = {p: SK.for_stage(runner, B, p, B.ops[-1:]) for p in parts_b} if rep_mode else {}
    held = {p: [] for p in parts_b}          # repartition pieces no sink could take (run at the end)

    def chunks():
        for p in parts_a:
            for t in ST._chunks(splan, p, dev, vctx_a[p]):
                yield p, t
    it = chunks()
    proto = None
    pending = None
    rounds, sent_rows, recv_rows = 0, 0, 0
    stats = EXC.ExchangeStats()
    t0 = time.perf_counter()
    wait_s = 0.0

    def fold(ex):
        nonlocal recv_rows, wait_s
        tw = time.perf_counter()
        got = ex.finish()
        wait_s += time.perf_counter() - tw
        for i, q in enumerate(parts_b):
            pieces = [lst[i] for lst in got if len(lst) > i and lst[i].n]
            if not pieces:
                continue
            tab = DeviceTable.concat(pieces) if len(pieces) > 1 else pieces[0]
            recv_rows += tab.n
            if not rep_mode:
                aggs[q].add_partial(tab)
                continue
            data = tab
            for op in B.ops[:-1]:                 # B's record-wise operators on the round's rows
                data = runner._run_op(op, [data], vctx_b[q], B)
            if held[q] or outs[q] is None or not outs[q].add(data):
                if outs[q] is not None and outs[q].started:
                    raise RuntimeError("streamed repartition: a round could not be written like the others")
                held[q].append(data)

    fold_err = None

    def agree(err, have, where):
        # one small tensor collective per round: every rank's status and whether it had a chunk;
        # a rank whose round failed stops every rank alike (no rank left inside an exchange)
        st = shuffle.gang_status(err is None, have, w)
        bad = [r for r, (ok, _) in enumerate(st) if not ok]
        if bad:
            from ..errors import GangAgreementError
            for sk in outs.values():
                if sk is not None:
                    sk.abort()
            raise GangAgreementError(f"streamed shuffle: rank(s) {bad} failed in {where}"
                                     + (f" ({type(err).__name__}: {err})" if err is not None else ""), ranks=bad) \
                from err
        return st

    while True:
        err, sends, item = fold_err, None, None
        try:
            item = next(it, None) if err is None else None
            if item is not None:
                p, t = item
                data = t
                for op in splan["pre"]:
                    data = runner._run_op(op, [data], vctx_a[p], A)
                part = data if rep_mode else runner._run_op(splan["agg"], [data], vctx_a[p], A)
                ported = runner._run_op(splan["rest"][0], [part], vctx_a[p], A)
                if not isinstance(ported, Ported) or not isinstance(ported.table, DeviceTable):
                    raise NotTraceable("streamed shuffle: the partial rows left the device")
                sends = [[ported.port(q) for q in owned[r]] for r in range(W)]
                proto = ported.port(0).slice(0, 0)
                sent_rows += ported.table.n
        except Exception as e:  # noqa: BLE001
            err = e
        st = agree(err, int(item is not None), f"round {rounds}")
        if not any(v for _, v in st):
            break
        if sends is None:
            # this rank's chunks are done: empty pieces of its layout (or none before its first)
            sends = [[proto for _ in owned[r]] for r in range(W)] if proto is not None else [[] for _ in range(W)]
        ex = EXC.exchange_start(w, sends, stats, arena=arena)   # queued; round r-1 is folded meanwhile
        if pending is not None:
            try:
                fold(pending)
            except Exception as e:  # noqa: BLE001  (agreed at the next round)
                fold_err = e
        pending = ex
        rounds += 1
    if pending is not None:
        try:
            fold(pending)
        except Exception as e:  # noqa: BLE001
            fold_err = e
    agree(fold_err, 0, "the last fold")
    t1 = time.perf_counter()
    out, written = {}, 0
    for q in parts_b:
        if rep_mode:
            sk = outs[q]
            if sk is not None and sk.started:
                value, nb = sk.finish()
            else:
                tabs = [x for x in held[q] if x is not None]
                if not tabs and proto is not None:
                    data = proto
                    for op in B.ops[:-1]:
                        data = runner._run_op(op, [data], vctx_b[q], B)
                    tabs = [data]
                value = DeviceTable.concat(tabs) if len(tabs) > 1 else (tabs[0] if tabs else [])
                value, nb = runner._run_op(B.ops[-1], [value], vctx_b[q], B), 0
            out[q] = value
            written += nb or 0
            continue
        value, nb = SA.finish(runner, B, q, vctx_b[q], aggs[q], True, B.ops[1:])
        out[q] = value
        written += nb or 0
    st = [a.stats for a in aggs.values()]
    runner.stream_stats[(B.id, me)] = dict(
        kind="streamed shuffle", mode="repartition" if rep_mode else "aggregation", rounds=rounds, sent_rows=sent_rows, received_rows=recv_rows,
        exchanged_GB=round((stats.bytes_sent + stats.bytes_received) / 2e9, 3), collectives=stats.collectives,
        exchange_wait_s=round(wait_s, 3), stream_s=round(t1 - t0, 3), finish_s=round(time.perf_counter() - t1, 3),
        spilled_bytes=sum(x.get("spilled_bytes", 0) for x in st), combines=sum(x.get("combines", 0) for x in st),
        dense_state=any("dense_state_GB" in x for x in st), budget_bytes=lay["budget"],
        held_batches=sum(x.get("held_batches", 0) for x in st),
        result="streamed to the output store" if written else "concatenated in HBM", result_bytes=written)
    return out

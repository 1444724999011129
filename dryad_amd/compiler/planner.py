"""Query planner: query DAG -> physical stage plan.

Reference: LinqToDryad/DryadLinqQueryGen.cs.  The phases are kept:

  Phase 0  SimpleRewriter (Where push-down)                          (:274)
  Phase 1  visit every operator and emit physical nodes with partition/order/distinct properties;
           strategies: decomposable GroupBy with partial aggregation (:2007-2359), two-phase
           sampling range partition (:2362-2474), OrderBy (:2476), hash/merge join with
           co-partitioning (:1419-1609), Take/Skip (:2546), Apply homomorphic / left-homomorphic /
           merged (:2925-3027), Fork (:3083), indexed operators through partition offsets
           (CreateOffset :1225-1248), Tee for shared sub-queries (:305-387)
  Phase 2  pipeline fusion of pointwise single-consumer nodes into one vertex ("SuperNode",
           DryadLinqQueryNode.cs:523-638)                                  (:391-456)
  Phase 3  id assignment and plan emission (JSON in place of the XML plan) (:634-701)
"""
from __future__ import annotations

import itertools
from dataclasses import dataclass, field

from .. import types as T
from ..attributes import is_expensive, is_homomorphic, is_left_homomorphic
from ..errors import DryadLinqException, ErrorCode
from ..query import QNode, _NOSEED
from .datasetinfo import DataSetInfo, OrderInfo, PartitionInfo, PartitionType
from .decomposition import decompose
from .plan import Plan, Stage, StageInput
from .rewriter import rewrite

SAMPLE_RATE = 0.001          # DryadLinqSampler.cs:38-39
SAMPLE_SEED = 314159


def _identity(x):
    return x


_identity._dryad_key_name = "identity"


def _pair_key(kv):
    return kv[0]


@dataclass
class PNode:
    """A physical node under construction (becomes a Stage after fusion)."""
    name: str
    partitions: int
    inputs: list = field(default_factory=list)        # StageInput with .src = PNode
    ops: list = field(default_factory=list)
    out_ports: int = 1
    info: DataSetInfo = field(default_factory=DataSetInfo)
    dtype: object = None
    output: dict | None = None
    consumers: int = 0
    explain: list = field(default_factory=list)
    fusable: bool = True
    dynamic_manager: str | None = None
    gang: bool = False
    id: int = -1


class Planner:
    def __init__(self, ctx, roots: list):
        self.ctx = ctx
        self.roots = roots
        self.P = ctx.num_partitions
        self.memo: dict = {}
        self.nodes: list = []
        self.outputs: list = []
        self.seps_nodes: dict = {}        # id -> separator PNode of each sampled range partition

    # ------------------------------------------------------------------ node helpers
    def _new(self, name, partitions, inputs=(), ops=(), info=None, out_ports=1, dtype=None) -> PNode:
        n = PNode(name, partitions, list(inputs), list(ops), out_ports, info or DataSetInfo(PartitionInfo.random(partitions)),
                  dtype)
        for i in n.inputs:
            i.src.consumers += 1
        self.nodes.append(n)
        return n

    def pointwise(self, src: PNode, name, ops, info=None, port=0, dtype=None) -> PNode:
        return self._new(name, src.partitions, [StageInput(src, "pointwise", port)], ops,
                         info or DataSetInfo(PartitionInfo.random(src.partitions)), dtype=dtype)

    def merge_one(self, src: PNode, name, ops=(), port=0, merge_sort=None, dtype=None) -> PNode:
        if src.partitions == 1 and not ops and port == 0:
            return src
        info = DataSetInfo(PartitionInfo.random(1), src.info.order if merge_sort else None, src.info.distinct
                           if src.partitions == 1 else False)
        return self._new(name, 1, [StageInput(src, "merge", port, merge_sort=merge_sort)], ops, info, dtype=dtype)

    def hash_shuffle(self, src: PNode, key, comparer, n, name="HashPartition", dtype=None) -> PNode:
        part = self.pointwise(src, name, [dict(op="hash_partition", key=key, comparer=comparer, count=n,
                                               explain=f"hash_partition(n={n})")])
        part.out_ports = n
        info = DataSetInfo(PartitionInfo.hash(key, n, comparer))
        m = self._new("Merge", n, [StageInput(part, "cross")], [], info, dtype=dtype or src.dtype)
        m.gang = True
        return m

    def range_shuffle(self, src: PNode, key, comparer, descending, n, separators=None, name="RangePartition",
                      seps_node: PNode | None = None):
        """Range partition (two-phase sampling unless ``separators`` are given).  ``seps_node``:
        reuse another data set's sampled separators (co-range partitioning for a join / set
        operation against a range-partitioned input, DryadLinqQueryGen.cs:1487-1512)."""
        if seps_node is not None:
            part = self._new(name, src.partitions, [StageInput(src, "pointwise"), StageInput(seps_node, "broadcast")],
                             [dict(op="range_partition", key=key, comparer=comparer, descending=descending,
                                   separators=None, count=n, keep_ties=True,
                                   explain=f"range_partition(n={n}, separators of stage '{seps_node.name}')")])
            part.out_ports = n
            info = DataSetInfo(PartitionInfo.range(key, n, None, descending, comparer, origin=part.ops[-1],
                                                   seps_id=id(seps_node)))
            m = self._new("Merge", n, [StageInput(part, "cross")], [], info, dtype=src.dtype)
            m.gang = True
            return m
        if separators is not None:
            n = len(separators) + 1
            part = self.pointwise(src, name, [dict(op="range_partition", key=key, comparer=comparer,
                                                   descending=descending, separators=list(separators), count=n,
                                                   explain=f"range_partition(separators={len(separators)})")])
        else:
            # two-phase sampling (DryadLinqSampler): sample per partition -> one vertex picks n-1 separators
            samp = self.pointwise(src, "Sample", [dict(op="sample", key=key, rate=SAMPLE_RATE, seed=SAMPLE_SEED,
                                                       explain=f"sample(rate={SAMPLE_RATE})")])
            seps = self.merge_one(samp, "Separators", [dict(op="separators", count=n, comparer=comparer,
                                                            descending=descending,
                                                            explain=f"choose {n - 1} separators")])
            part = self._new(name, src.partitions, [StageInput(src, "pointwise"), StageInput(seps, "broadcast")],
                             [dict(op="range_partition", key=key, comparer=comparer, descending=descending,
                                   separators=None, count=n, explain=f"range_partition(n={n}, sampled)")])
            self.seps_nodes[id(seps)] = seps
        part.out_ports = n
        info = DataSetInfo(PartitionInfo.range(key, n, separators, descending, comparer, origin=part.ops[-1],
                                               seps_id=id(seps) if separators is None else None))
        m = self._new("Merge", n, [StageInput(part, "cross")], [], info, dtype=src.dtype)
        m.gang = True
        return m

    def range_like(self, src: PNode, key, part: PartitionInfo) -> PNode:
        """Range-partition ``src`` by ``key`` exactly like the range-partitioned data set ``part``
        (its explicit separators, or its sampled separator stage broadcast to this partition step)."""
        part.rely_on_colocation()
        if part.separators is not None:
            return self.range_shuffle(src, key, part.comparer, part.descending, part.count, list(part.separators))
        seps = self.seps_nodes.get(part.seps_id)
        if seps is None:
            return None
        return self.range_shuffle(src, key, part.comparer, part.descending, part.count, seps_node=seps)

    def local_sort(self, src: PNode, key, cmp, desc, why) -> PNode:
        """Sort each partition (no shuffle): the other side of an ordered (merge) operator."""
        n = self.pointwise(src, "OrderBy", [dict(op="sort", key=key, comparer=cmp, descending=desc,
                                                 explain=f"sort{' desc' if desc else ''} per partition ({why})")],
                           DataSetInfo(src.info.partition, OrderInfo(key, cmp, desc), src.info.distinct),
                           dtype=src.dtype)
        return n

    # ------------------------------------------------------------------ compile
    def compile(self) -> Plan:
        outs = []
        for r in self.roots:
            r2 = rewrite(r)
            pn = self.visit(r2)
            outs.append(pn)
        self._fuse()
        self._cleanup()
        stages = self._emit()
        plan = Plan(stages, [s.id for s in stages if s.is_output], self._globals())
        return plan

    def _globals(self):
        c = self.ctx
        return {"DryadLinqVersion": c.ClientVersion(), "ClusterName": c.PlatformKind.value,
                "MinimumComputeNodes": c.JobMinNodes, "MaximumComputeNodes": c.JobMaxNodes,
                "IntermediateDataCompression": c.IntermediateDataCompressionScheme.name,
                "EnableSpeculativeDuplication": c.EnableSpeculativeDuplication, "QueryName": c.JobFriendlyName,
                "DefaultPartitionCount": self.P}

    def visit(self, q: QNode) -> PNode:
        hit = self.memo.get(q.id)
        if hit is not None:
            return hit
        pn = self._visit(q)
        if q.dtype is not None and q.op in ("FromEnumerable", "FromStore", "Table", "ToStore"):
            pn.dtype = q.dtype
        self.memo[q.id] = pn
        return pn

    def _visit(self, q: QNode) -> PNode:
        a = q.args
        op = q.op
        fn = getattr(self, "v_" + op, None)
        if fn is None:
            raise DryadLinqException(ErrorCode.OperatorNotSupported, f"operator {op} is not supported")
        return fn(q, a)

    # ------------------------------------------------------------------ inputs / outputs
    def v_FromEnumerable(self, q, a):
        data = a["data"]
        P = max(1, self.P)
        chunks = [data[(len(data) * i) // P:(len(data) * (i + 1)) // P] for i in range(P)]
        return self._new("Input", P, [], [dict(op="enumerable", chunks=chunks, dtype=q.dtype,
                                              explain=f"FromEnumerable({len(data)} records)")],
                         DataSetInfo(PartitionInfo.random(P)), dtype=q.dtype)

    def v_FromStore(self, q, a):
        from ..io.providers import provider_for
        uri = a["uri"]
        n, size = provider_for(uri).stream_info(uri)
        return self._new("Input", n, [], [dict(op="read", uri=uri, dtype=q.dtype, deserializer=a.get("deserializer"),
                                               explain=f"read {uri}")],
                         DataSetInfo(PartitionInfo.random(n)), dtype=q.dtype)

    v_Table = v_FromStore

    def v_ToStore(self, q, a):
        src = self.visit(q.sources[0])
        out = self.pointwise(src, "Output", [dict(op="output", uri=a["uri"], dtype=q.dtype or src.dtype,
                                                  serializer=a.get("serializer"), explain=f"write {a['uri']}")],
                             info=src.info, dtype=q.dtype or src.dtype)
        out.output = dict(uri=a["uri"], delete_if_exists=a.get("delete_if_exists", False), temp=a.get("_temp", False),
                          qnode=q)
        out.fusable = True
        self.outputs.append(out)
        return out

    # ------------------------------------------------------------------ pointwise operators
    def _indexed(self, src: PNode, name, op):
        counts = self.pointwise(src, "Count", [dict(op="count", explain="count")])
        offs = self.merge_one(counts, "Offsets", [dict(op="offsets", explain="partition offsets")])
        return self._new(name, src.partitions, [StageInput(src, "pointwise"), StageInput(offs, "broadcast")],
                         [op], DataSetInfo(PartitionInfo.random(src.partitions)))

    def v_Where(self, q, a):
        src = self.visit(q.sources[0])
        if a.get("indexed"):
            return self._indexed(src, "Where", dict(op="where_idx", fn=a["predicate"], explain="where (indexed)"))
        info = DataSetInfo(src.info.partition, src.info.order, src.info.distinct)
        return self.pointwise(src, "Where", [dict(op="where", fn=a["predicate"], explain="where")], info, dtype=src.dtype)

    def v_Select(self, q, a):
        src = self.visit(q.sources[0])
        if a.get("indexed"):
            return self._indexed(src, "Select", dict(op="select_idx", fn=a["selector"], explain="select (indexed)"))
        return self.pointwise(src, "Select", [dict(op="select", fn=a["selector"], explain="select")])

    def v_SelectMany(self, q, a):
        src = self.visit(q.sources[0])
        if a.get("indexed"):
            return self._indexed(src, "SelectMany", dict(op="select_many_idx", fn=a["selector"],
                                                         result=a.get("result_selector"), explain="select_many (indexed)"))
        return self.pointwise(src, "SelectMany", [dict(op="select_many", fn=a["selector"], result=a.get("result_selector"),
                                                       explain="select_many")])

    def v_Take(self, q, a):
        src = self.visit(q.sources[0])
        n = a["count"]
        if src.partitions == 1:
            return self.pointwise(src, "Take", [dict(op="take", count=n, explain=f"take({n})")], src.info, dtype=src.dtype)
        local = self.pointwise(src, "Take", [dict(op="take", count=n, explain=f"take({n}) per partition")], dtype=src.dtype)
        return self.merge_one(local, "Take", [dict(op="take", count=n, explain=f"take({n})")], dtype=src.dtype)

    def _merged_unary(self, q, name, op):
        src = self.visit(q.sources[0])
        m = self.merge_one(src, name, [op], dtype=src.dtype)
        if m is src:
            return self.pointwise(src, name, [op], src.info, dtype=src.dtype)
        return m

    def v_Skip(self, q, a):
        return self._merged_unary(q, "Skip", dict(op="skip", count=a["count"], explain=f"skip({a['count']})"))

    def v_TakeWhile(self, q, a):
        return self._merged_unary(q, "TakeWhile", dict(op="take_while", fn=a["predicate"], indexed=a.get("indexed"),
                                                       explain="take_while"))

    def v_SkipWhile(self, q, a):
        return self._merged_unary(q, "SkipWhile", dict(op="skip_while", fn=a["predicate"], indexed=a.get("indexed"),
                                                       explain="skip_while"))

    def v_Reverse(self, q, a):
        return self._merged_unary(q, "Reverse", dict(op="reverse", explain="reverse"))

    def v_SlidingWindow(self, q, a):
        return self._merged_unary(q, "SlidingWindow", dict(op="sliding_window", fn=a["func"], window=a["window_size"],
                                                           explain=f"sliding_window({a['window_size']})"))

    # ------------------------------------------------------------------ ordering / partitioning
    def v_OrderBy(self, q, a):
        src = self.visit(q.sources[0])
        key, cmp, desc = a["key_selector"], a.get("comparer"), a.get("descending", False)
        sort_op = dict(op="sort", key=key, comparer=cmp, descending=desc, explain="sort" + (" desc" if desc else ""))
        if src.info.order is not None and src.info.order.is_ordered_by(key, cmp, desc) and (
                src.partitions == 1 or src.info.partition.kind == PartitionType.RANGE and src.info.partition.is_partitioned_by(key)):
            return src
        if src.partitions == 1 and not self.ctx._props.get("ExchangeOneRank", False):
            info = DataSetInfo(PartitionInfo.random(1), OrderInfo(key, cmp, desc), src.info.distinct)
            return self.pointwise(src, "OrderBy", [sort_op], info, dtype=src.dtype)
        if src.info.partition.kind == PartitionType.RANGE and src.info.partition.is_partitioned_by(key, cmp) \
                and src.info.partition.descending == desc:
            shuffled = src
        else:
            shuffled = self.range_shuffle(src, key, cmp, desc, src.partitions)
        info = DataSetInfo(shuffled.info.partition, OrderInfo(key, cmp, desc))
        node = self.pointwise(shuffled, "OrderBy", [sort_op], info, dtype=src.dtype)
        return node

    def v_RangePartition(self, q, a):
        src = self.visit(q.sources[0])
        n = a.get("count") or src.partitions
        return self.range_shuffle(src, a["key_selector"], a.get("comparer"), a.get("descending", False), n,
                                  a.get("separators"))

    def v_HashPartition(self, q, a):
        src = self.visit(q.sources[0])
        n = a.get("count") or self.P
        m = self.hash_shuffle(src, a["key_selector"], a.get("comparer"), n)
        if a.get("result_selector") is not None:
            return self.pointwise(m, "Select", [dict(op="select", fn=a["result_selector"], explain="result_selector")],
                                  DataSetInfo(PartitionInfo.random(n)))
        return m

    def _assume(self, src, info, name):
        n = self.pointwise(src, name, [], info, dtype=src.dtype)
        return n

    def v_AssumeHashPartition(self, q, a):
        src = self.visit(q.sources[0])
        return self._assume(src, DataSetInfo(PartitionInfo.hash(a["key_selector"], src.partitions, a.get("comparer")),
                                             src.info.order, src.info.distinct), "AssumeHashPartition")

    def v_AssumeRangePartition(self, q, a):
        src = self.visit(q.sources[0])
        return self._assume(src, DataSetInfo(PartitionInfo.range(a["key_selector"], src.partitions, a.get("separators"),
                                                                 a.get("descending", False), a.get("comparer")),
                                             src.info.order, src.info.distinct), "AssumeRangePartition")

    def v_AssumeOrderBy(self, q, a):
        src = self.visit(q.sources[0])
        return self._assume(src, DataSetInfo(src.info.partition, OrderInfo(a["key_selector"], a.get("comparer"),
                                                                           a.get("descending", False)),
                                             src.info.distinct), "AssumeOrderBy")

    # ------------------------------------------------------------------ GroupBy
    def v_GroupBy(self, q, a):
        src = self.visit(q.sources[0])
        key, elem, res, cmp = a["key_selector"], a.get("element_selector"), a.get("result_selector"), a.get("comparer")
        gb = dict(op="group_by", key=key, elem=elem, result=res, comparer=cmp, explain="group_by")
        if src.info.partition.is_partitioned_by(key, cmp):
            d = decompose(res, elem) if res is not None else None
            if d is not None:   # lets the device run it as one partial-aggregation pass
                gb["decomp"] = d
            why = []
            if src.partitions > 1:
                why.append(f"input {src.info.partition.kind.value}-partitioned by the key: no shuffle")
            if src.info.order is not None and src.info.order.is_ordered_by(key, cmp, src.info.order.descending):
                # OrderedGroupBy (DryadLinqQueryGen.cs:2098-2100): groups are runs of the sorted input
                gb.update(op="ordered_group_by", explain="ordered_group_by (runs of equal keys, no hash table / sort)")
                why.append("input ordered by the key: no sort")
            n = self.pointwise(src, "GroupBy", [gb], DataSetInfo(src.info.partition if res is None else
                                                                 PartitionInfo.random(src.partitions)))
            n.explain.extend(why)
            return n
        n = self.P
        d = decompose(res, elem) if res is not None else None
        if d is not None:
            partial = self.pointwise(src, "GroupBy", [dict(op="group_partial", key=key, decomp=d, comparer=cmp,
                                                           explain=f"group_partial({len(d.aggs)} aggregates)")])
            shuffled = self.hash_shuffle(partial, _pair_key, cmp, n)
            final = self.pointwise(shuffled, "GroupBy", [dict(op="group_final", decomp=d, comparer=cmp,
                                                              explain="group_final (RecursiveAccumulate+FinalReduce)")])
            final.explain.append("decomposable GroupBy: partial aggregation before the shuffle")
            return final
        shuffled = self.hash_shuffle(src, key, cmp, n)
        return self.pointwise(shuffled, "GroupBy", [gb], DataSetInfo(PartitionInfo.random(n)))

    # ------------------------------------------------------------------ joins
    def _copartition(self, left: PNode, lkey, right: PNode, rkey, cmp):
        n = self.P
        lp, rp = left.info.partition, right.info.partition
        if lp.kind == PartitionType.HASH and rp.kind == PartitionType.HASH and lp.is_partitioned_by(lkey, cmp) \
                and rp.is_partitioned_by(rkey, cmp) and lp.count == rp.count:
            return left, right
        if lp.count == 1 and rp.count == 1:
            return left, right
        if lp.kind == PartitionType.HASH and lp.is_partitioned_by(lkey, cmp):
            n = lp.count
            return left, self.hash_shuffle(right, rkey, cmp, n)
        if rp.kind == PartitionType.HASH and rp.is_partitioned_by(rkey, cmp):
            n = rp.count
            return self.hash_shuffle(left, lkey, cmp, n), right
        return self.hash_shuffle(left, lkey, cmp, n), self.hash_shuffle(right, rkey, cmp, n)

    def _binary(self, name, l, r, op, info=None):
        return self._new(name, l.partitions, [StageInput(l, "pointwise"), StageInput(r, "pointwise")], [op],
                         info or DataSetInfo(PartitionInfo.random(l.partitions)))

    def _range_copartition(self, left: PNode, lkey, right: PNode, rkey, cmp):
        """Co-partition against a side that is already range-partitioned by its key (reference
        DryadLinqQueryGen.cs:1487-1512: range-distribute the other side with the same
        separators); None when neither side is."""
        lp, rp = left.info.partition, right.info.partition
        if lp.count > 1 and lp.kind == PartitionType.RANGE and lp.is_partitioned_by(lkey, cmp):
            if rp.kind == PartitionType.RANGE and rp.is_partitioned_by(rkey, cmp) and lp.is_same_partition(rp):
                return left, right, "both sides range-partitioned alike: no shuffle"
            r2 = self.range_like(right, rkey, lp)
            if r2 is not None:
                return left, r2, "outer range-partitioned by the key: inner range-partitioned alike"
        if rp.count > 1 and rp.kind == PartitionType.RANGE and rp.is_partitioned_by(rkey, cmp):
            l2 = self.range_like(left, lkey, rp)
            if l2 is not None:
                return l2, right, "inner range-partitioned by the key: outer range-partitioned alike"
        return None

    def _ordered_pair(self, l: PNode, lkey, r: PNode, rkey, cmp):
        """Merge strategy (DryadLinqQueryGen.cs:1574-1597, 1862-1880): when either side is sorted by
        its key within each partition, sort the other side per partition -> (l, r, note) or None."""
        lo, ro = l.info.order, r.info.order
        if lo is not None and lo.is_ordered_by(lkey, cmp, lo.descending):
            if ro is None or not ro.is_ordered_by(rkey, cmp, lo.descending):
                return l, self.local_sort(r, rkey, cmp, lo.descending, "merge with the ordered outer"), \
                    "outer ordered by the key: inner sorted per partition, merge"
            return l, r, "both sides ordered by the key: merge (no sort)"
        if ro is not None and ro.is_ordered_by(rkey, cmp, ro.descending):
            return self.local_sort(l, lkey, cmp, ro.descending, "merge with the ordered inner"), r, \
                "inner ordered by the key: outer sorted per partition, merge"
        return None

    def v_Join(self, q, a, group=False):
        outer = self.visit(q.sources[0])
        inner = self.visit(q.sources[1])
        ok, ik, cmp = a["outer_key"], a["inner_key"], a.get("comparer")
        notes = []
        co = self._range_copartition(outer, ok, inner, ik, cmp)
        if co is not None:
            l, r, why = co
            notes.append(why)
        else:
            l, r = self._copartition(outer, ok, inner, ik, cmp)
        od = self._ordered_pair(l, ok, r, ik, cmp) if cmp is None else None
        if od is not None:
            l, r, why = od
            notes.append(why)
            kind = "merge_group_join" if group else "merge_join"
        else:
            kind = "hash_group_join" if group else "hash_join"
        jop = dict(op=kind, outer_key=ok, inner_key=ik, result=a["result_selector"], comparer=cmp, explain=kind)
        if od is not None:
            jop["descending"] = l.info.order.descending
        node = self._binary("GroupJoin" if group else "Join", l, r, jop)
        node.explain.extend(notes)
        return node

    def v_GroupJoin(self, q, a):
        return self.v_Join(q, a, group=True)

    # ------------------------------------------------------------------ set operations
    def v_Distinct(self, q, a):
        src = self.visit(q.sources[0])
        cmp = a.get("comparer")
        if src.info.distinct:
            return src
        ordered = cmp is None and src.info.order is not None and \
            src.info.order.is_ordered_by(_identity, None, src.info.order.descending)
        if src.info.partition.is_partitioned_by(_identity, cmp):
            op = dict(op="ordered_distinct", comparer=cmp, explain="ordered_distinct (drop adjacent duplicates)") \
                if ordered else dict(op="distinct", comparer=cmp, explain="distinct")
            n = self.pointwise(src, "Distinct", [op], DataSetInfo(src.info.partition, src.info.order, True),
                               dtype=src.dtype)
            if src.partitions > 1:
                n.explain.append("input partitioned by the record: no shuffle")
            return n
        partial = self.pointwise(src, "Distinct", [dict(op="distinct", comparer=cmp, explain="distinct (partial)")],
                                 DataSetInfo(src.info.partition, src.info.order, True), dtype=src.dtype)
        sh = self.hash_shuffle(partial, _identity, cmp, self.P)
        info = DataSetInfo(sh.info.partition, None, True)
        return self.pointwise(sh, "Distinct", [dict(op="distinct", comparer=cmp, explain="distinct")], info,
                              dtype=src.dtype)

    def _setop(self, q, a, kind):
        l = self.visit(q.sources[0])
        r = self.visit(q.sources[1])
        cmp = a.get("comparer")
        if kind == "union":
            l = self.pointwise(l, "Distinct", [dict(op="distinct", comparer=cmp, explain="distinct (partial)")],
                               DataSetInfo(l.info.partition, l.info.order, True), dtype=l.dtype)
            r = self.pointwise(r, "Distinct", [dict(op="distinct", comparer=cmp, explain="distinct (partial)")],
                               DataSetInfo(r.info.partition, r.info.order, True), dtype=r.dtype)
        notes = []
        co = self._range_copartition(l, _identity, r, _identity, cmp)
        if co is not None:
            l2, r2, why = co
            notes.append(why)
        else:
            l2, r2 = self._copartition(l, _identity, r, _identity, cmp)
        od = self._ordered_pair(l2, _identity, r2, _identity, cmp) if cmp is None else None
        order = None
        if od is not None:
            l2, r2, why = od
            notes.append(why)
            order = l2.info.order
            op = dict(op="ordered_" + kind, comparer=cmp, descending=order.descending,
                      explain=f"ordered_{kind} (merge of sorted inputs)")
        else:
            op = dict(op=kind, comparer=cmp, explain=kind)
        info = DataSetInfo(l2.info.partition, order, True)
        node = self._binary(kind.capitalize(), l2, r2, op, info)
        node.explain.extend(notes)
        return node

    def v_Union(self, q, a):
        return self._setop(q, a, "union")

    def v_Intersect(self, q, a):
        return self._setop(q, a, "intersect")

    def v_Except(self, q, a):
        return self._setop(q, a, "except")

    def v_Concat(self, q, a):
        l = self.visit(q.sources[0])
        r = self.visit(q.sources[1])
        return self._new("Concat", l.partitions + r.partitions,
                         [StageInput(l, "offset", 0, 0), StageInput(r, "offset", 0, l.partitions)],
                         [dict(op="concat", explain="concat")],
                         DataSetInfo(PartitionInfo.random(l.partitions + r.partitions)), dtype=l.dtype)

    def v_Zip(self, q, a):
        l = self.merge_one(self.visit(q.sources[0]), "Merge")
        r = self.merge_one(self.visit(q.sources[1]), "Merge")
        return self._binary("Zip", l, r, dict(op="zip", fn=a["result_selector"], explain="zip"),
                            DataSetInfo(PartitionInfo.random(1)))

    # ------------------------------------------------------------------ aggregates (-> one record)
    def _aggregate(self, q, a, kind):
        src = self.visit(q.sources[0])
        spec = dict(kind=kind, **{k: v for k, v in a.items() if k in ("predicate", "selector", "comparer", "value",
                                                                         "seed", "func", "result_selector")})
        if kind == "Aggregate":
            func = a["func"]
            assoc = getattr(func, "_dryad_associative", None)
            if assoc is None:
                m = self.merge_one(src, "Aggregate")
                return self.pointwise(m, "Aggregate", [dict(op="aggregate_seq", spec=spec, explain="aggregate")],
                                      DataSetInfo(PartitionInfo.random(1)), dtype=None) if m is src else \
                    self._append(m, dict(op="aggregate_seq", spec=spec, explain="aggregate"))
            spec["assoc"] = assoc()
        partial = self.pointwise(src, kind, [dict(op="agg_partial", spec=spec, explain=f"{kind} (partial)")])
        partial = self._aggregation_tree(partial, kind, spec)
        if partial.partitions <= 1:
            return self._append(partial, dict(op="agg_final", spec=spec, explain=f"{kind} (final)"))
        final = self.merge_one(partial, kind, [dict(op="agg_final", spec=spec, explain=f"{kind} (final)")])
        if kind == "Aggregate" and is_expensive(a["func"]):
            # expensive associative fold: a dynamic aggregation tree (DryadLinqQueryNode.cs:2866-2871
            # FullAggregator, AggregationLevels = 2; DrDynamicAggregateManager) folds the partials
            # of each machine (GPU rank) into one before the final vertex
            final.dynamic_manager = "FullAggregator"
            final.explain.append("dynamic FullAggregator: partials folded per rank before the final aggregate")
        return final

    def _aggregation_tree(self, partial: PNode, kind, spec) -> PNode:
        """Aggregation tree (reference DrDynamicAggregateManager, GraphBuilder.cs:633-703;
        DryadLinqApplication.cs:173-175: at most 150 inputs per aggregation vertex, groups of
        32): while more partials than the fan-in limit would meet in one merge vertex, insert a
        level of combine vertices, each folding one group of partials into one partial.  The
        groups are dynamic: the process executor regroups the partials by their actual output sizes
        against ``AggregateThreshold`` once they exist (runtime/aggmanager.py); the static groups
        of ``AggregationTreeGroup`` bound the number of combine vertices."""
        max_in = int(self.ctx._props.get("AggregationTreeMaxInputs") or 150)
        group = int(self.ctx._props.get("AggregationTreeGroup") or 32)
        level = 0
        while partial.partitions > max_in and group > 1:
            level += 1
            n = -(-partial.partitions // group)
            partial = self._new(f"{kind}Combine", n, [StageInput(partial, "group", group=group, dynamic=True)],
                                [dict(op="agg_combine", spec=spec, explain=f"{kind} (combine, tree level {level})")],
                                DataSetInfo(PartitionInfo.random(n)))
        return partial

    def _append(self, node: PNode, op):
        node.ops.append(op)
        return node

    def v_Count(self, q, a):
        return self._aggregate(q, a, "Count")

    def v_LongCount(self, q, a):
        return self._aggregate(q, a, "Count")

    def v_Sum(self, q, a):
        return self._aggregate(q, a, "Sum")

    def v_Min(self, q, a):
        return self._aggregate(q, a, "Min")

    def v_Max(self, q, a):
        return self._aggregate(q, a, "Max")

    def v_Average(self, q, a):
        return self._aggregate(q, a, "Average")

    def v_Any(self, q, a):
        return self._aggregate(q, a, "Any")

    def v_All(self, q, a):
        return self._aggregate(q, a, "All")

    def v_Contains(self, q, a):
        return self._aggregate(q, a, "Contains")

    def v_First(self, q, a):
        return self._aggregate(q, a, "First")

    def v_FirstOrDefault(self, q, a):
        return self._aggregate(q, a, "FirstOrDefault")

    def v_Last(self, q, a):
        return self._aggregate(q, a, "Last")

    def v_LastOrDefault(self, q, a):
        return self._aggregate(q, a, "LastOrDefault")

    def v_Single(self, q, a):
        return self._aggregate(q, a, "Single")

    def v_SingleOrDefault(self, q, a):
        return self._aggregate(q, a, "SingleOrDefault")

    def v_Aggregate(self, q, a):
        return self._aggregate(q, a, "Aggregate")

    def v_SequenceEqual(self, q, a):
        l = self.merge_one(self.visit(q.sources[0]), "Merge")
        r = self.merge_one(self.visit(q.sources[1]), "Merge")
        return self._binary("SequenceEqual", l, r, dict(op="sequence_equal", comparer=a.get("comparer"),
                                                        explain="sequence_equal"), DataSetInfo(PartitionInfo.random(1)))

    # ------------------------------------------------------------------ Apply / Fork
    def v_Apply(self, q, a):
        srcs = [self.visit(s) for s in q.sources]
        func = a["func"]
        per_part = a.get("per_partition") or is_homomorphic(func)
        first_only = a.get("first_only") or is_left_homomorphic(func)
        op = dict(op="apply", fn=func, multi=a.get("multi", False), explain="apply" + (" per partition" if per_part else ""),
                  in_dtypes=[s.dtype for s in q.sources])
        if per_part:
            lead = srcs[0]
            inputs = [StageInput(lead, "pointwise")]
            for s in srcs[1:]:
                if first_only:
                    inputs.append(StageInput(s, "broadcast"))
                else:
                    if s.partitions != lead.partitions:
                        raise DryadLinqException(ErrorCode.HomomorphicApplyNeedsSamePartitionCount,
                                                 "homomorphic Apply needs inputs with the same partition count")
                    inputs.append(StageInput(s, "pointwise"))
            if len(inputs) == 1:
                n = self.pointwise(lead, "Apply", [op])
                n.fusable = not is_expensive(func)
                return n
            return self._new("Apply", lead.partitions, inputs, [op], DataSetInfo(PartitionInfo.random(lead.partitions)))
        merged = [self.merge_one(s, "Merge") for s in srcs]
        if len(merged) == 1:
            m = merged[0]
            if m is srcs[0]:
                return self.pointwise(m, "Apply", [op], DataSetInfo(PartitionInfo.random(1)))
            return self._append(m, op)
        return self._new("Apply", 1, [StageInput(m, "pointwise") for m in merged], [op],
                         DataSetInfo(PartitionInfo.random(1)))

    def v_ApplyWithPartitionIndex(self, q, a):
        src = self.visit(q.sources[0])
        return self.pointwise(src, "Apply", [dict(op="apply_index", fn=a["func"], explain="apply_with_partition_index")])

    def v_Fork(self, q, a):
        src = self.visit(q.sources[0])
        keys = a.get("keys")
        ports = len(keys) if keys is not None else 3
        n = self.pointwise(src, "Fork", [dict(op="fork", mapper=a["mapper"], keys=keys, per_record=a.get("per_record"),
                                              explain=f"fork({ports} outputs)")])
        n.out_ports = ports
        return n

    def v_ForkPort(self, q, a):
        fork = self.visit(q.sources[0])
        return self.pointwise(fork, "ForkOutput", [], DataSetInfo(PartitionInfo.random(fork.partitions)),
                              port=a["port"])

    # ------------------------------------------------------------------ Phase 2: fusion
    def _fuse(self):
        changed = True
        while changed:
            changed = False
            for n in list(self.nodes):
                if len(n.inputs) != 1:
                    continue
                inp = n.inputs[0]
                p = inp.src
                if inp.kind != "pointwise" or inp.port != 0 or p.out_ports != 1 or p.consumers != 1:
                    continue
                if not n.fusable or not p.fusable or p.output is not None:
                    continue
                if p.partitions != n.partitions:
                    continue
                # fuse n into p
                p.ops.extend(n.ops)
                p.out_ports = n.out_ports
                p.info = n.info
                p.dtype = n.dtype
                p.output = n.output
                p.fusable = n.fusable
                p.gang = p.gang or n.gang
                p.explain.extend(n.explain)
                if n.name not in ("Merge", "ForkOutput") and n.ops:
                    p.name = n.name if p.name in ("Merge", "Input", "ForkOutput") else p.name + "+" + n.name
                p.consumers = n.consumers
                for m in self.nodes:
                    for i in m.inputs:
                        if i.src is n:
                            i.src = p
                self.outputs = [p if o is n else o for o in self.outputs]
                self.nodes.remove(n)
                changed = True
                break

    # ------------------------------------------------------------------ Phase 3: cleanup + emit
    def _cleanup(self):
        """Remove useless Merge nodes (DryadLinqQueryGen.cs:474-500): an op-less Merge between a
        CrossProduct exchange and its only consumer (a Join / set operation / Apply with several
        inputs, which fusion could not absorb) -> the consumer takes the exchange directly (one
        vertex hop and one HBM channel fewer per partition)."""
        for n in list(self.nodes):
            if n.ops or n.output is not None or len(n.inputs) != 1 or n.inputs[0].kind != "cross":
                continue
            cons = [(m, i) for m in self.nodes for i in m.inputs if i.src is n]
            if len(cons) != 1 or n in self.outputs:
                continue
            m, i = cons[0]
            if i.kind != "pointwise" or i.port != 0 or m.partitions != n.partitions:
                continue
            src_in = n.inputs[0]
            i.src, i.kind, i.port, i.merge_sort = src_in.src, "cross", src_in.port, src_in.merge_sort
            m.gang = True
            m.explain.append(f"{n.name} vertex elided: the exchange feeds this stage directly")
            self.nodes.remove(n)


    def _emit(self) -> list:
        # topological order (inputs before consumers)
        order, seen = [], set()

        def go(n):
            if id(n) in seen:
                return
            seen.add(id(n))
            for i in n.inputs:
                go(i.src)
            order.append(n)
        for n in self.nodes:
            go(n)
        for k, n in enumerate(order):
            n.id = k
        stages = []
        for n in order:
            ins = [StageInput(i.src.id, i.kind, i.port, i.offset, i.merge_sort, i.group, getattr(i, "dynamic", False)) for i in n.inputs]
            ops = n.ops if n.ops else [dict(op="identity", explain="merge")]
            st = Stage(n.id, n.name, n.partitions, ins, ops, n.out_ports, n.dtype, n.info,
                       dict(n.output) if n.output else None, n.dynamic_manager, explain=list(n.explain), gang=n.gang)
            stages.append(st)
        return stages


def compile_queries(ctx, queries) -> Plan:
    roots = [q.node if hasattr(q, "node") else q for q in queries]
    return Planner(ctx, roots).compile()

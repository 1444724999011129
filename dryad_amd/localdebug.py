"""LocalDebug executor: evaluates a query DAG with LINQ-to-Objects semantics (the oracle).

Reference: DryadLinqLocalProvider + ``IsLocalDebugSource`` short-circuit
(LinqToDryad/DryadLinqQueryable.cs:41-44, DryadLinqQuery.cs) — with ``context.LocalDebug = true``
queries never compile to a DAG; they run in-process over IEnumerables.  Here the same DAG that
the planner compiles is interpreted node by node with ``dryad_amd.enumerable``.
"""
from __future__ import annotations

from . import enumerable as E
from .errors import DryadLinqException, ErrorCode
from .query import _NOSEED, QNode

SCALAR_OPS = {"Count", "LongCount", "Any", "All", "Contains", "SequenceEqual", "First", "FirstOrDefault", "Last",
              "LastOrDefault", "Single", "SingleOrDefault", "Sum", "Min", "Max", "Average", "Aggregate"}


def eval_scalar(op: str, src, a: dict, other=None):
    if op in ("Count", "LongCount"):
        return E.Count(src, a.get("predicate"))
    if op == "Any":
        return E.Any(src, a.get("predicate"))
    if op == "All":
        return E.All(src, a["predicate"])
    if op == "Contains":
        return E.Contains(src, a["value"], a.get("comparer"))
    if op == "SequenceEqual":
        return E.SequenceEqual(src, other, a.get("comparer"))
    if op in ("First", "FirstOrDefault", "Last", "LastOrDefault", "Single", "SingleOrDefault"):
        return getattr(E, op)(src, a.get("predicate"))
    if op == "Sum":
        return E.Sum(src, a.get("selector"))
    if op == "Min":
        return E.Min(src, a.get("selector"), a.get("comparer"))
    if op == "Max":
        return E.Max(src, a.get("selector"), a.get("comparer"))
    if op == "Average":
        return E.Average(src, a.get("selector"))
    if op == "Aggregate":
        seed = a.get("seed", _NOSEED)
        return E.Aggregate(src, E._NO if seed is _NOSEED else seed, a["func"], a.get("result_selector"))
    raise DryadLinqException(ErrorCode.OperatorNotSupported, op)


class LocalEvaluator:
    def __init__(self, ctx):
        self.ctx = ctx
        self.cache: dict = {}

    def eval(self, node: QNode) -> list:
        hit = self.cache.get(node.id)
        if hit is not None:
            return hit
        out = self._eval(node)
        if not isinstance(out, list):
            out = list(out)
        self.cache[node.id] = out
        return out

    def _eval(self, n: QNode):
        a = n.args
        op = n.op
        srcs = [self.eval(s) for s in n.sources] if op not in ("Fork",) else None
        s0 = srcs[0] if srcs else None
        if op == "FromEnumerable":
            return list(a["data"])
        if op in ("FromStore", "Table"):
            from .io.providers import provider_for
            return list(provider_for(a["uri"]).read_all(a["uri"], n.dtype))
        if op == "Where":
            return E.Where(s0, a["predicate"], a.get("indexed", False))
        if op == "Select":
            return E.Select(s0, a["selector"], a.get("indexed", False))
        if op == "SelectMany":
            return E.SelectMany(s0, a["selector"], a.get("result_selector"), a.get("indexed", False))
        if op in ("Take", "Skip"):
            return getattr(E, op)(s0, a["count"])
        if op in ("TakeWhile", "SkipWhile"):
            return getattr(E, op)(s0, a["predicate"], a.get("indexed", False))
        if op == "OrderBy":
            return E.OrderBy(s0, a["key_selector"], a.get("comparer"), a.get("descending", False))
        if op == "GroupBy":
            return E.GroupBy(s0, a["key_selector"], a.get("element_selector"), a.get("result_selector"),
                             a.get("comparer"))
        if op == "Join":
            return E.Join(s0, srcs[1], a["outer_key"], a["inner_key"], a["result_selector"], a.get("comparer"))
        if op == "GroupJoin":
            return E.GroupJoin(s0, srcs[1], a["outer_key"], a["inner_key"], a["result_selector"], a.get("comparer"))
        if op == "Distinct":
            return E.Distinct(s0, a.get("comparer"))
        if op == "Concat":
            return E.Concat(s0, srcs[1])
        if op in ("Union", "Intersect", "Except"):
            return getattr(E, op)(s0, srcs[1], a.get("comparer"))
        if op == "Zip":
            return E.Zip(s0, srcs[1], a["result_selector"])
        if op == "Reverse":
            return E.Reverse(s0)
        if op == "HashPartition":
            return E.HashPartition(s0, a["key_selector"], a.get("comparer"), a.get("count"), a.get("result_selector"))
        if op in ("RangePartition", "AssumeHashPartition", "AssumeRangePartition", "AssumeOrderBy", "Merge",
                  "Tee"):
            return s0
        if op == "Apply":
            f = a["func"]
            from .attributes import is_device_function
            if is_device_function(f):
                from .device_udf import call_on_records
                return call_on_records(f, srcs, [s.dtype for s in n.sources], bool(a.get("multi")))
            if a.get("multi"):
                return f([s0] + srcs[1:]) if len(srcs) > 1 else f([s0])
            return f(*srcs)
        if op == "ApplyWithPartitionIndex":
            return E.ApplyWithPartitionIndex(s0, a["func"])
        if op == "SlidingWindow":
            return E.SlidingWindow(s0, a["func"], a["window_size"])
        if op == "ForkPort":
            outs = self._fork(n.sources[0])
            return outs[a["port"]]
        if op == "Fork":
            return self._fork(n)
        if op == "ToStore":
            self.ctx._write_local_store(n, s0)
            return s0
        if op in SCALAR_OPS:
            return [eval_scalar(op, s0, a, srcs[1] if len(srcs) > 1 else None)]
        raise DryadLinqException(ErrorCode.OperatorNotSupported, f"operator {op} is not supported in LocalDebug")

    def _fork(self, fnode: QNode):
        key = ("fork", fnode.id)
        hit = self.cache.get(key)
        if hit is not None:
            return hit
        src = self.eval(fnode.sources[0])
        a = fnode.args
        if a.get("keys") is not None:
            outs = E.Fork(src, a["mapper"], a["keys"])
        elif a.get("per_record"):
            outs = E.Fork(src, lambda seq: (a["mapper"](x) for x in seq))
        else:
            outs = E.Fork(src, a["mapper"])
        self.cache[key] = outs
        return outs

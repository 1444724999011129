"""Object-level vertex operator library (the CPU path of every plan op).

Reference: LinqToDryad/DryadLinqVertex.cs — Where/Select/SelectMany (:74-192), Sort/MergeSort
(:293-423), GroupBy hash with partial/full accumulation (:437-583), HashJoin/MergeJoin/
HashGroupJoin/MergeGroupJoin (:852-1162), set operations (:1232-1597), aggregates (:1673-4697),
Apply (:4726-4785), HashPartition (:4788-4907: port = (hash & 0x7FFFFFFF) % nPorts), RangePartition
(:4909-5151, binary search of separators), Fork (:5153-5300).  Each op takes the list of input
streams (lists) and the vertex context and returns a list, or a list of port lists.

Hashing must agree across worker processes (Python's str hash is salted per process), so
partitioners use ``stable_hash``: FNV-1a over a canonical byte encoding, or the user comparer's
``GetHashCode``.
"""
from __future__ import annotations

import bisect
import dataclasses
import functools
import heapq
import itertools
import math
import random
import struct
from collections import OrderedDict

from .. import enumerable as E
from ..errors import DryadLinqException, ErrorCode


class VertexContext:
    def __init__(self, partition=0, partitions=1, vertex_id=0, version=0, stage=None, job=None):
        self.partition = partition
        self.partitions = partitions
        self.vertex_id = vertex_id
        self.version = version
        self.stage = stage
        self.job = job
        self.outputs_written = []


# ---------------------------------------------------------------------------------------------
_FNV_OFF = 0xCBF29CE484222325
_FNV_PRIME = 0x100000001B3
_M64 = (1 << 64) - 1


def _fnv(b: bytes, h=_FNV_OFF) -> int:
    for x in b:
        h = ((h ^ x) * _FNV_PRIME) & _M64
    return h


def stable_hash(k, comparer=None) -> int:
    """Process-independent 32-bit hash (non-negative)."""
    if comparer is not None:
        h = comparer.GetHashCode(k) if hasattr(comparer, "GetHashCode") else comparer.hash(k)
        return h & 0x7FFFFFFF
    return _h(k) & 0x7FFFFFFF


def _h(k) -> int:
    if k is None:
        return 0
    if isinstance(k, bool):
        return 1 if k else 0
    if isinstance(k, int):
        x = k & _M64
        x ^= x >> 33
        x = (x * 0xFF51AFD7ED558CCD) & _M64
        x ^= x >> 33
        return x
    if isinstance(k, float):
        # mirrored bit for bit by the device partitioner (csrc/kernels/stablehash.hip)
        if k != k:
            return _fnv(struct.pack("<Q", 0x7FF8000000000000))
        if math.isfinite(k) and abs(k) < 2**63 and k == int(k):
            return _h(int(k))
        return _fnv(struct.pack("<d", k))
    if isinstance(k, str):
        return _fnv(k.encode("utf-8", "surrogatepass"))
    if isinstance(k, (bytes, bytearray, memoryview)):
        return _fnv(bytes(k))
    if isinstance(k, (tuple, list)):
        h = 0x345678
        for x in k:
            h = ((h ^ _h(x)) * 1000003) & _M64
        return h
    if dataclasses.is_dataclass(k):
        return _h(tuple(getattr(k, f.name) for f in dataclasses.fields(k)))
    if hasattr(k, "Line"):
        return _h(k.Line)
    return _fnv(repr(k).encode())


def hash_port(k, n, comparer=None) -> int:
    return stable_hash(k, comparer) % n


# ---------------------------------------------------------------------------------------------
def _one(inputs):
    return inputs[0] if len(inputs) == 1 else [x for s in inputs for x in s]


def op_enumerable(op, inputs, v):
    return list(op["chunks"][v.partition])


def op_read(op, inputs, v):
    from ..io.providers import provider_for
    uri = op["uri"]
    p = provider_for(uri)
    if op.get("deserializer") is not None and hasattr(p, "read_partition_bytes"):
        import io
        return list(op["deserializer"](io.BytesIO(p.read_partition_bytes(uri, v.partition))))
    return p.read_partition(uri, v.partition, op.get("dtype"))


def op_identity(op, inputs, v):
    return _one(inputs)


def op_concat(op, inputs, v):
    return [x for s in inputs for x in s]


def op_where(op, inputs, v):
    f = op["fn"]
    return [x for x in _one(inputs) if f(x)]


def op_select(op, inputs, v):
    f = op["fn"]
    return [f(x) for x in _one(inputs)]


def op_select_many(op, inputs, v):
    return list(E.SelectMany(_one(inputs), op["fn"], op.get("result")))


def _offset(inputs, v):
    offs = inputs[1]
    return offs[v.partition] if v.partition < len(offs) else 0


def op_where_idx(op, inputs, v):
    base, f = _offset(inputs, v), op["fn"]
    return [x for i, x in enumerate(inputs[0]) if f(x, base + i)]


def op_select_idx(op, inputs, v):
    base, f = _offset(inputs, v), op["fn"]
    return [f(x, base + i) for i, x in enumerate(inputs[0])]


def op_select_many_idx(op, inputs, v):
    base, f, r = _offset(inputs, v), op["fn"], op.get("result")
    out = []
    for i, x in enumerate(inputs[0]):
        for y in f(x, base + i):
            out.append(r(x, y) if r is not None else y)
    return out


def op_take(op, inputs, v):
    return _one(inputs)[: max(0, op["count"])]


def op_skip(op, inputs, v):
    return _one(inputs)[max(0, op["count"]):]


def op_take_while(op, inputs, v):
    return list(E.TakeWhile(_one(inputs), op["fn"], op.get("indexed", False)))


def op_skip_while(op, inputs, v):
    return list(E.SkipWhile(_one(inputs), op["fn"], op.get("indexed", False)))


def op_reverse(op, inputs, v):
    return list(reversed(_one(inputs)))


def op_sliding_window(op, inputs, v):
    return list(E.SlidingWindow(_one(inputs), op["fn"], op["window"]))


def op_sort(op, inputs, v):
    return E.OrderBy(_one(inputs), op["key"], op.get("comparer"), op.get("descending", False))


def op_count(op, inputs, v):
    return [len(_one(inputs))]


def op_offsets(op, inputs, v):
    counts = _one(inputs)
    return E.Offsets(counts)


# ---------------------------------------------------------------------------------------------
# GroupBy
def op_group_by(op, inputs, v):
    return E.GroupBy(_one(inputs), op["key"], op.get("elem"), op.get("result"), op.get("comparer"))


def op_group_partial(op, inputs, v):
    """Local partial aggregation: (key, [acc per aggregate]) per distinct key (hash accumulation,
    reference ParallelHashGroupByPartialAccumulate :5718)."""
    key, d, cmp = op["key"], op["decomp"], op.get("comparer")
    wrap = E.eq_wrapper(cmp)
    table = OrderedDict()
    for x in _one(inputs):
        k = key(x)
        wk = wrap(k)
        cur = table.get(wk)
        if cur is None:
            table[wk] = (k, d.seed(x))
        else:
            table[wk] = (cur[0], d.accumulate(cur[1], x))
    return list(table.values())


def op_group_final(op, inputs, v):
    d, cmp = op["decomp"], op.get("comparer")
    wrap = E.eq_wrapper(cmp)
    table = OrderedDict()
    for k, accs in _one(inputs):
        wk = wrap(k)
        cur = table.get(wk)
        table[wk] = (k, accs) if cur is None else (cur[0], d.combine(cur[1], accs))
    return [d.final(k, accs) for k, accs in table.values()]


# ---------------------------------------------------------------------------------------------
# Joins (two inputs: outer, inner)
def op_hash_join(op, inputs, v):
    return list(E.Join(inputs[0], inputs[1], op["outer_key"], op["inner_key"], op["result"], op.get("comparer")))


def op_hash_group_join(op, inputs, v):
    return list(E.GroupJoin(inputs[0], inputs[1], op["outer_key"], op["inner_key"], op["result"], op.get("comparer")))


def _merge_join_iter(outer, inner, ok, ik, cmp, descending=False):
    c0 = E.compare_fn(cmp)
    c = (lambda a, b: -c0(a, b)) if descending else c0
    j = 0
    n = len(inner)
    for x in outer:
        kx = ok(x)
        while j < n and c(ik(inner[j]), kx) < 0:
            j += 1
        m = j
        group = []
        while m < n and c(ik(inner[m]), kx) == 0:
            group.append(inner[m])
            m += 1
        yield x, group


def op_merge_join(op, inputs, v):
    out, r = [], op["result"]
    for x, group in _merge_join_iter(inputs[0], inputs[1], op["outer_key"], op["inner_key"], op.get("comparer"),
                                     op.get("descending", False)):
        for y in group:
            out.append(r(x, y))
    return out


def op_merge_group_join(op, inputs, v):
    r = op["result"]
    return [r(x, E.LinqList(g)) for x, g in _merge_join_iter(inputs[0], inputs[1], op["outer_key"], op["inner_key"],
                                                  op.get("comparer"), op.get("descending", False))]


# ---------------------------------------------------------------------------------------------
# set operations
def op_distinct(op, inputs, v):
    return list(E.Distinct(_one(inputs), op.get("comparer")))


def op_union(op, inputs, v):
    return list(E.Union(inputs[0], inputs[1], op.get("comparer")))


def op_intersect(op, inputs, v):
    return list(E.Intersect(inputs[0], inputs[1], op.get("comparer")))


def op_except(op, inputs, v):
    return list(E.Except(inputs[0], inputs[1], op.get("comparer")))


# ordered strategies (reference OrderedGroupBy / OrderedDistinct / Ordered* set operations,
# DryadLinqVertex.cs:586-760, 1232-1597): the inputs are sorted by the key (record), so groups
# are runs and set operations are merges; no hash table, output stays sorted
def op_ordered_group_by(op, inputs, v):
    key, elem, res, cmp = op["key"], op.get("elem"), op.get("result"), op.get("comparer")
    wrap = E.eq_wrapper(cmp)
    out, cur, wk = [], None, None
    for x in _one(inputs):
        k = key(x)
        w = wrap(k)
        if cur is None or w != wk:
            cur, wk = E.Grouping(k), w
            out.append(cur)
        cur.append(elem(x) if elem is not None else x)
    return out if res is None else [res(g.Key, g) for g in out]


def op_ordered_distinct(op, inputs, v):
    out, last, first = [], None, True
    for x in _one(inputs):
        if first or x != last:
            out.append(x)
        last, first = x, False
    return out


def _ordered_merge(a, b, descending):
    """(x, in_a, in_b) over the distinct records of two sorted sequences, in their order."""
    c0 = E.compare_fn(None)
    c = (lambda x, y: -c0(x, y)) if descending else c0
    a, b = op_ordered_distinct(None, [a], None), op_ordered_distinct(None, [b], None)
    i = j = 0
    while i < len(a) or j < len(b):
        if j >= len(b) or (i < len(a) and c(a[i], b[j]) < 0):
            yield a[i], True, False
            i += 1
        elif i >= len(a) or c(a[i], b[j]) > 0:
            yield b[j], False, True
            j += 1
        else:
            yield a[i], True, True
            i += 1
            j += 1


def op_ordered_union(op, inputs, v):
    return [x for x, _, _ in _ordered_merge(inputs[0], inputs[1], op.get("descending", False))]


def op_ordered_intersect(op, inputs, v):
    return [x for x, ia, ib in _ordered_merge(inputs[0], inputs[1], op.get("descending", False)) if ia and ib]


def op_ordered_except(op, inputs, v):
    return [x for x, ia, ib in _ordered_merge(inputs[0], inputs[1], op.get("descending", False)) if ia and not ib]


def op_zip(op, inputs, v):
    return list(E.Zip(inputs[0], inputs[1], op["fn"]))


def op_sequence_equal(op, inputs, v):
    return [E.SequenceEqual(inputs[0], inputs[1], op.get("comparer"))]


# ---------------------------------------------------------------------------------------------
# Aggregates: partial per partition -> final on one vertex (two-stage, DryadLinqQueryGen.cs:3384-3395)
_NONE = ("__none__",)


def op_agg_partial(op, inputs, v):
    s = op["spec"]
    k = s["kind"]
    src = _one(inputs)
    pred, sel = s.get("predicate"), s.get("selector")
    if k == "Count":
        return [E.Count(src, pred)]
    if k == "Sum":
        return [E.Sum(src, sel)]
    if k in ("Min", "Max"):
        vals = [x for x in (src if sel is None else (sel(x) for x in src)) if x is not None]
        if not vals:
            return [_NONE]
        return [E.Min(vals, None, s.get("comparer")) if k == "Min" else E.Max(vals, None, s.get("comparer"))]
    if k == "Average":
        tot, n = 0, 0
        for x in (src if sel is None else (sel(x) for x in src)):
            if x is not None:
                tot += x
                n += 1
        return [(tot, n)]
    if k == "Any":
        return [E.Any(src, pred)]
    if k == "All":
        return [E.All(src, pred)]
    if k == "Contains":
        return [E.Contains(src, s["value"], s.get("comparer"))]
    if k in ("First", "FirstOrDefault", "Last", "LastOrDefault"):
        matches = [x for x in src if pred is None or pred(x)]
        if not matches:
            return [(False, None)]
        return [(True, matches[0] if k.startswith("First") else matches[-1])]
    if k in ("Single", "SingleOrDefault"):
        matches = [x for x in src if pred is None or pred(x)]
        return [(len(matches), matches[0] if matches else None)]
    if k == "Aggregate":
        assoc = s["assoc"]
        acc = assoc.Seed()
        for x in src:
            acc = assoc.RecursiveAccumulate(acc, x)
        return [acc]
    raise DryadLinqException(ErrorCode.OperatorNotSupported, f"aggregate {k}")


def op_agg_final(op, inputs, v):
    s = op["spec"]
    k = s["kind"]
    parts = _one(inputs)
    if k == "Count":
        return [sum(parts)]
    if k == "Sum":
        tot = 0
        for p in parts:
            tot = tot + p
        return [tot]
    if k in ("Min", "Max"):
        vals = [p for p in parts if p != _NONE]
        if not vals:
            raise E.InvalidOperationException("Sequence contains no elements")
        return [E.Min(vals, None, s.get("comparer")) if k == "Min" else E.Max(vals, None, s.get("comparer"))]
    if k == "Average":
        tot = sum(p[0] for p in parts)
        n = sum(p[1] for p in parts)
        if n == 0:
            raise E.InvalidOperationException("Sequence contains no elements")
        return [tot / n]
    if k in ("Any", "Contains"):
        return [any(parts)]
    if k == "All":
        return [all(parts)]
    if k in ("First", "FirstOrDefault"):
        for found, x in parts:
            if found:
                return [x]
        if k == "First":
            raise E.InvalidOperationException("Sequence contains no matching element")
        return [None]
    if k in ("Last", "LastOrDefault"):
        for found, x in reversed(parts):
            if found:
                return [x]
        if k == "Last":
            raise E.InvalidOperationException("Sequence contains no matching element")
        return [None]
    if k in ("Single", "SingleOrDefault"):
        n = sum(c for c, _ in parts)
        if n > 1:
            raise E.InvalidOperationException("Sequence contains more than one matching element")
        if n == 0:
            if k == "Single":
                raise E.InvalidOperationException("Sequence contains no matching element")
            return [None]
        return [next(x for c, x in parts if c)]
    if k == "Aggregate":
        assoc = s["assoc"]
        acc = assoc.Seed()
        for p in parts:
            acc = assoc.RecursiveAccumulate(acc, p)
        r = s.get("result_selector")
        return [r(acc) if r else acc]
    raise DryadLinqException(ErrorCode.OperatorNotSupported, f"aggregate {k}")


def op_agg_combine(op, inputs, v):
    """Fold a group of partial aggregates into ONE partial of the same shape (aggregation-tree
    interior vertex: RecursiveAccumulate without FinalReduce)."""
    s = op["spec"]
    k = s["kind"]
    parts = _one(inputs)
    if k in ("Count", "Sum"):
        tot = 0
        for p in parts:
            tot = tot + p
        return [tot]
    if k in ("Min", "Max"):
        vals = [p for p in parts if p != _NONE]
        if not vals:
            return [_NONE]
        return [E.Min(vals, None, s.get("comparer")) if k == "Min" else E.Max(vals, None, s.get("comparer"))]
    if k == "Average":
        return [(sum(p[0] for p in parts), sum(p[1] for p in parts))]
    if k in ("Any", "Contains"):
        return [any(parts)]
    if k == "All":
        return [all(parts)]
    if k in ("First", "FirstOrDefault", "Last", "LastOrDefault"):
        found = [p for p in parts if p[0]]
        if not found:
            return [(False, None)]
        return [found[0] if k.startswith("First") else found[-1]]
    if k in ("Single", "SingleOrDefault"):
        n = sum(c for c, _ in parts)
        x = next((x for c, x in parts if c), None)
        return [(n, x)]
    if k == "Aggregate":
        assoc = s["assoc"]
        acc = assoc.Seed()
        for p in parts:
            acc = assoc.RecursiveAccumulate(acc, p)
        return [acc]
    raise DryadLinqException(ErrorCode.OperatorNotSupported, f"aggregate {k}")


def op_aggregate_seq(op, inputs, v):
    from ..localdebug import eval_scalar
    s = op["spec"]
    return [eval_scalar("Aggregate", _one(inputs), s)]


# ---------------------------------------------------------------------------------------------
# partitioners
def op_hash_partition(op, inputs, v):
    n, key, cmp = op["count"], op["key"], op.get("comparer")
    ports = [[] for _ in range(n)]
    for x in _one(inputs):
        ports[hash_port(key(x), n, cmp)].append(x)
    return ports


def op_sample(op, inputs, v):
    """Per-partition Bernoulli sample of keys at `rate`, seeded by the vertex id so re-execution
    reproduces it; all keys when fewer than 10 would be drawn (DryadLinqSampler.cs:38-106)."""
    src = _one(inputs)
    key = op["key"]
    rate = op.get("rate", 0.001)
    if len(src) * rate < 10:
        return [key(x) for x in src]
    rng = random.Random(op.get("seed", 314159) * 1000003 + v.partition)
    return [key(x) for x in src if rng.random() < rate]


def op_separators(op, inputs, v):
    """Reservoir (<=1M keys, seed 314159), sort, pick count-1 evenly spaced separators
    (DryadLinqSampler.cs:129-246)."""
    keys = _one(inputs)
    cap = 1 << 20
    if len(keys) > cap:
        rng = random.Random(314159)
        res = keys[:cap]
        for i in range(cap, len(keys)):
            j = rng.randint(0, i)
            if j < cap:
                res[j] = keys[i]
        keys = res
    n = op["count"]
    keys = E.OrderBy(keys, lambda k: k, op.get("comparer"), op.get("descending", False))
    if not keys:
        return []
    return [keys[(len(keys) * j) // n] for j in range(1, n)]


def op_range_partition(op, inputs, v):
    n, key, cmp, desc = op["count"], op["key"], op.get("comparer"), op.get("descending", False)
    seps = op.get("separators")
    if seps is None:
        seps = inputs[1] if len(inputs) > 1 else []
    src = inputs[0]
    ports = [[] for _ in range(n)]
    if not seps:
        ports[0].extend(src)
        return ports
    c = E.compare_fn(cmp)
    kf = functools.cmp_to_key((lambda a, b: -c(a, b)) if desc else c)
    ks = [kf(s) for s in seps]
    for x in src:
        p = bisect.bisect_left(ks, kf(key(x)))   # count of separators strictly before the key
        ports[min(p, n - 1)].append(x)
    return ports


# ---------------------------------------------------------------------------------------------
def op_apply(op, inputs, v):
    f = op["fn"]
    from ..attributes import is_device_function
    if is_device_function(f):
        from ..device_udf import call_on_records
        return call_on_records(f, list(inputs), op.get("in_dtypes") or [], bool(op.get("multi")))
    if op.get("multi"):
        res = f(list(inputs))
    else:
        res = f(*inputs)
    return list(res)


def op_apply_index(op, inputs, v):
    return list(op["fn"](_one(inputs), v.partition))


def op_fork(op, inputs, v):
    src = _one(inputs)
    keys = op.get("keys")
    if keys is not None:
        return E.Fork(src, op["mapper"], keys)
    if op.get("per_record"):
        m = op["mapper"]
        return E.Fork(src, lambda seq: (m(x) for x in seq))
    return E.Fork(src, op["mapper"])


def op_output(op, inputs, v):
    # the runtime writes the stream to the output table's part file (commit-by-rename)
    return _one(inputs)


OPS = {k[3:]: fn for k, fn in list(globals().items()) if k.startswith("op_")}


def run_program(ops: list, inputs: list, vctx: VertexContext):
    """Execute a stage's vertex program; returns a list of output port streams."""
    data = None
    for i, op in enumerate(ops):
        fn = OPS.get(op["op"])
        if fn is None:
            raise DryadLinqException(ErrorCode.OperatorNotSupported, f"vertex op {op['op']}")
        data = fn(op, inputs if i == 0 else [data], vctx)
    return data

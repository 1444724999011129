"""The DryadLINQ query surface: lazy ``Query`` objects with the reference operator set.

Reference: LinqToDryad/DryadLinqQueryable.cs (operator surface, :39-4322), DryadLinqQuery.cs
(query objects: plain data / data-backed / expression states, :37-692), MultiQueryable.cs
(multi-output Fork results).  Each operator appends a ``QNode`` to an immutable expression DAG;
nothing runs until a terminal operator (scalar aggregate, enumeration, ``Submit``/``SubmitAndWait``).

Python has no static overloads, so C# overloads are resolved by keyword arguments and, where the
C# signatures differ only in delegate shape, by the lambda's arity (``Select(lambda x, i: ...)`` is
the indexed overload, like ``Select<T,R>(Func<T,int,R>)``).  Every operator also has a snake_case
alias (``q.select(...)``).
"""
from __future__ import annotations

import inspect
import itertools
from typing import Any, Callable

from .errors import DryadLinqException, ErrorCode

_ids = itertools.count(1)


def nparams(f) -> int:
    try:
        sig = inspect.signature(f)
    except (TypeError, ValueError):
        return 1
    n = 0
    for p in sig.parameters.values():
        if p.kind in (p.POSITIONAL_ONLY, p.POSITIONAL_OR_KEYWORD) and p.default is p.empty:
            n += 1
        elif p.kind == p.VAR_POSITIONAL:
            return 99
    return n


class QNode:
    """One operator application in the query DAG."""
    __slots__ = ("id", "op", "sources", "args", "dtype", "port", "__weakref__")

    def __init__(self, op: str, sources=(), args: dict | None = None, dtype=None, port: int | None = None):
        self.id = next(_ids)
        self.op = op
        self.sources = tuple(sources)
        self.args = dict(args or {})
        self.dtype = dtype
        self.port = port

    def __repr__(self):
        return f"QNode#{self.id}({self.op})"

    def walk(self):
        """All nodes reachable from this one (post-order, each once)."""
        seen, out = set(), []

        def go(n):
            if n.id in seen:
                return
            seen.add(n.id)
            for s in n.sources:
                go(s)
            out.append(n)
        go(self)
        return out


def _is_eq_comparer(o) -> bool:
    return o is not None and (hasattr(o, "Equals") and hasattr(o, "GetHashCode") or
                              hasattr(o, "equals") and hasattr(o, "hash"))


def _is_cmp_comparer(o) -> bool:
    return o is not None and (hasattr(o, "Compare") or (callable(o) and nparams(o) == 2))


class Query:
    """IQueryable<T>: a lazy, immutable DryadLINQ query bound to a context."""

    def __init__(self, ctx, node: QNode):
        self._ctx = ctx
        self._node = node

    # ----------------------------------------------------------------- plumbing
    @property
    def context(self):
        return self._ctx

    @property
    def node(self) -> QNode:
        return self._node

    @property
    def dtype(self):
        return self._node.dtype

    def _q(self, op, sources=None, dtype=None, **args) -> "Query":
        srcs = [self._node] + [s._node if isinstance(s, Query) else s for s in (sources or [])]
        return Query(self._ctx, QNode(op, srcs, args, dtype))

    def _other(self, other) -> QNode:
        if isinstance(other, Query):
            if other._ctx is not self._ctx and not self._ctx._compatible(other._ctx):
                raise DryadLinqException(ErrorCode.MustStartFromContext,
                                         "queries from different DryadLinqContexts cannot be combined")
            return other._node
        # a plain Python iterable: lift it
        return self._ctx.FromEnumerable(list(other))._node

    def __repr__(self):
        return f"<DryadLinq Query {self._node.op}#{self._node.id}>"

    def __iter__(self):
        return iter(self._ctx._enumerate(self))

    def ToList(self) -> list:
        return list(self)

    def ToArray(self) -> list:
        return list(self)

    def AsEnumerable(self):
        return iter(self)

    def ToDictionary(self, key_selector, element_selector=None) -> dict:
        out = {}
        for x in self:
            k = key_selector(x)
            if k in out:
                raise DryadLinqException(ErrorCode.TooManyItems, f"duplicate key {k!r}")
            out[k] = element_selector(x) if element_selector else x
        return out

    def ToLookup(self, key_selector, element_selector=None) -> dict:
        out = {}
        for x in self:
            out.setdefault(key_selector(x), []).append(element_selector(x) if element_selector else x)
        return out

    def Explain(self) -> str:
        return self._ctx.Explain(self)

    # ----------------------------------------------------------------- standard LINQ
    def Where(self, predicate: Callable) -> "Query":
        return self._q("Where", predicate=predicate, indexed=nparams(predicate) >= 2)

    def Select(self, selector: Callable) -> "Query":
        return self._q("Select", selector=selector, indexed=nparams(selector) >= 2)

    def SelectMany(self, collection_selector: Callable, result_selector: Callable | None = None) -> "Query":
        return self._q("SelectMany", selector=collection_selector, result_selector=result_selector,
                       indexed=nparams(collection_selector) >= 2)

    def LongWhere(self, predicate):
        return self._q("Where", predicate=predicate, indexed=True, long_index=True)

    def LongSelect(self, selector):
        return self._q("Select", selector=selector, indexed=True, long_index=True)

    def LongSelectMany(self, collection_selector, result_selector=None):
        return self._q("SelectMany", selector=collection_selector, result_selector=result_selector, indexed=True,
                       long_index=True)

    def LongTakeWhile(self, predicate):
        return self._q("TakeWhile", predicate=predicate, indexed=True, long_index=True)

    def LongSkipWhile(self, predicate):
        return self._q("SkipWhile", predicate=predicate, indexed=True, long_index=True)

    def Take(self, count: int):
        return self._q("Take", count=int(count))

    def Skip(self, count: int):
        return self._q("Skip", count=int(count))

    def TakeWhile(self, predicate):
        return self._q("TakeWhile", predicate=predicate, indexed=nparams(predicate) >= 2)

    def SkipWhile(self, predicate):
        return self._q("SkipWhile", predicate=predicate, indexed=nparams(predicate) >= 2)

    def OrderBy(self, key_selector, comparer=None):
        return self._q("OrderBy", key_selector=key_selector, comparer=comparer, descending=False)

    def OrderByDescending(self, key_selector, comparer=None):
        return self._q("OrderBy", key_selector=key_selector, comparer=comparer, descending=True)

    def ThenBy(self, *a, **k):
        raise DryadLinqException(ErrorCode.OperatorNotSupported, "ThenBy is not supported; use a composite key")

    def ThenByDescending(self, *a, **k):
        raise DryadLinqException(ErrorCode.OperatorNotSupported, "ThenByDescending is not supported")

    def DefaultIfEmpty(self, *a, **k):
        raise DryadLinqException(ErrorCode.OperatorNotSupported, "DefaultIfEmpty is not supported")

    def ElementAt(self, *a, **k):
        raise DryadLinqException(ErrorCode.OperatorNotSupported, "ElementAt is not supported")

    ElementAtOrDefault = ElementAt

    def OfType(self, *a, **k):
        raise DryadLinqException(ErrorCode.OperatorNotSupported, "OfType is not supported")

    def GroupBy(self, key_selector, element_selector=None, result_selector=None, comparer=None):
        # GroupBy(key, resultSelector(key, group)) overload: a 2-ary second argument
        if element_selector is not None and result_selector is None and nparams(element_selector) == 2 \
                and not _is_eq_comparer(element_selector):
            element_selector, result_selector = None, element_selector
        if _is_eq_comparer(element_selector):
            element_selector, comparer = None, element_selector
        if _is_eq_comparer(result_selector):
            result_selector, comparer = None, result_selector
        return self._q("GroupBy", key_selector=key_selector, element_selector=element_selector,
                       result_selector=result_selector, comparer=comparer)

    def Join(self, inner, outer_key_selector, inner_key_selector, result_selector, comparer=None):
        return Query(self._ctx, QNode("Join", [self._node, self._other(inner)],
                                      dict(outer_key=outer_key_selector, inner_key=inner_key_selector,
                                           result_selector=result_selector, comparer=comparer)))

    def GroupJoin(self, inner, outer_key_selector, inner_key_selector, result_selector, comparer=None):
        return Query(self._ctx, QNode("GroupJoin", [self._node, self._other(inner)],
                                      dict(outer_key=outer_key_selector, inner_key=inner_key_selector,
                                           result_selector=result_selector, comparer=comparer)))

    def Distinct(self, comparer=None):
        return self._q("Distinct", comparer=comparer)

    def Concat(self, other):
        return Query(self._ctx, QNode("Concat", [self._node, self._other(other)], {}, self.dtype))

    def Union(self, other, comparer=None):
        return Query(self._ctx, QNode("Union", [self._node, self._other(other)], dict(comparer=comparer), self.dtype))

    def Intersect(self, other, comparer=None):
        return Query(self._ctx, QNode("Intersect", [self._node, self._other(other)], dict(comparer=comparer),
                                      self.dtype))

    def Except(self, other, comparer=None):
        return Query(self._ctx, QNode("Except", [self._node, self._other(other)], dict(comparer=comparer),
                                      self.dtype))

    def Zip(self, other, result_selector):
        return Query(self._ctx, QNode("Zip", [self._node, self._other(other)], dict(result_selector=result_selector)))

    def Reverse(self):
        return self._q("Reverse", dtype=self.dtype)

    # ----------------------------------------------------------------- scalar operators (execute now)
    def _scalar(self, op, **args):
        return self._ctx._execute_scalar(Query(self._ctx, QNode(op, [self._node], args)))

    def _as_query(self, op, **args):
        return Query(self._ctx, QNode(op, [self._node], args))

    def Count(self, predicate=None):
        return self._scalar("Count", predicate=predicate)

    def LongCount(self, predicate=None):
        return self._scalar("LongCount", predicate=predicate)

    def Any(self, predicate=None):
        return self._scalar("Any", predicate=predicate)

    def All(self, predicate):
        return self._scalar("All", predicate=predicate)

    def Contains(self, value, comparer=None):
        return self._scalar("Contains", value=value, comparer=comparer)

    def SequenceEqual(self, other, comparer=None):
        return self._ctx._execute_scalar(Query(self._ctx, QNode("SequenceEqual", [self._node, self._other(other)],
                                                                dict(comparer=comparer))))

    def First(self, predicate=None):
        return self._scalar("First", predicate=predicate)

    def FirstOrDefault(self, predicate=None):
        return self._scalar("FirstOrDefault", predicate=predicate)

    def Last(self, predicate=None):
        return self._scalar("Last", predicate=predicate)

    def LastOrDefault(self, predicate=None):
        return self._scalar("LastOrDefault", predicate=predicate)

    def Single(self, predicate=None):
        return self._scalar("Single", predicate=predicate)

    def SingleOrDefault(self, predicate=None):
        return self._scalar("SingleOrDefault", predicate=predicate)

    def Sum(self, selector=None):
        return self._scalar("Sum", selector=selector)

    def Min(self, selector=None, comparer=None):
        return self._scalar("Min", selector=selector, comparer=comparer)

    def Max(self, selector=None, comparer=None):
        return self._scalar("Max", selector=selector, comparer=comparer)

    def Average(self, selector=None):
        return self._scalar("Average", selector=selector)

    def Aggregate(self, *args):
        seed, func, result = _aggregate_args(args)
        return self._scalar("Aggregate", seed=seed, func=func, result_selector=result)

    # ----------------------------------------------------------------- *AsQuery (lazy scalars)
    def AnyAsQuery(self, predicate=None):
        return self._as_query("Any", predicate=predicate)

    def AllAsQuery(self, predicate):
        return self._as_query("All", predicate=predicate)

    def CountAsQuery(self, predicate=None):
        return self._as_query("Count", predicate=predicate)

    def LongCountAsQuery(self, predicate=None):
        return self._as_query("LongCount", predicate=predicate)

    def ContainsAsQuery(self, value, comparer=None):
        return self._as_query("Contains", value=value, comparer=comparer)

    def SequenceEqualAsQuery(self, other, comparer=None):
        return Query(self._ctx, QNode("SequenceEqual", [self._node, self._other(other)], dict(comparer=comparer)))

    def FirstAsQuery(self, predicate=None):
        return self._as_query("First", predicate=predicate)

    def LastAsQuery(self, predicate=None):
        return self._as_query("Last", predicate=predicate)

    def SingleAsQuery(self, predicate=None):
        return self._as_query("Single", predicate=predicate)

    def MinAsQuery(self, selector=None, comparer=None):
        return self._as_query("Min", selector=selector, comparer=comparer)

    def MaxAsQuery(self, selector=None, comparer=None):
        return self._as_query("Max", selector=selector, comparer=comparer)

    def SumAsQuery(self, selector=None):
        return self._as_query("Sum", selector=selector)

    def AverageAsQuery(self, selector=None):
        return self._as_query("Average", selector=selector)

    def AggregateAsQuery(self, *args):
        seed, func, result = _aggregate_args(args)
        return self._as_query("Aggregate", seed=seed, func=func, result_selector=result)

    # ----------------------------------------------------------------- DryadLINQ partitioning
    def HashPartition(self, key_selector, *args, comparer=None, partition_count=None, result_selector=None):
        """HashPartition(keySel[, comparer][, partitionCount][, resultSelector]) (6 overloads)."""
        for a in args:
            if isinstance(a, int) and not isinstance(a, bool):
                partition_count = a
            elif _is_eq_comparer(a):
                comparer = a
            elif callable(a):
                result_selector = a
        if partition_count is not None and partition_count <= 0:
            raise ValueError(f"partitionCount must be positive, got {partition_count}")  # ArgumentOutOfRange
        return self._q("HashPartition", key_selector=key_selector, comparer=comparer, count=partition_count,
                       result_selector=result_selector, dtype=None if result_selector else self.dtype)

    def RangePartition(self, key_selector, *args, partition_count=None, is_descending=False, range_separators=None,
                       comparer=None):
        """RangePartition(keySel, [partitionCount|rangeSeparators], [comparer], [isDescending]) (9 overloads)."""
        for a in args:
            if isinstance(a, bool):
                is_descending = a
            elif isinstance(a, int):
                partition_count = a
            elif isinstance(a, (list, tuple)):
                range_separators = list(a)
            elif _is_cmp_comparer(a):
                comparer = a
        if partition_count is not None and partition_count <= 0:
            raise ValueError(f"partitionCount must be positive, got {partition_count}")  # ArgumentOutOfRange
        if range_separators is not None:
            _check_separators(range_separators, comparer, is_descending)
        return self._q("RangePartition", key_selector=key_selector, count=partition_count,
                       descending=bool(is_descending), separators=range_separators, comparer=comparer,
                       dtype=self.dtype)

    def AssumeHashPartition(self, key_selector, comparer=None):
        return self._q("AssumeHashPartition", key_selector=key_selector, comparer=comparer, dtype=self.dtype)

    def AssumeRangePartition(self, key_selector, *args, is_descending=False, range_separators=None, comparer=None):
        for a in args:
            if isinstance(a, bool):
                is_descending = a
            elif isinstance(a, (list, tuple)):
                range_separators = list(a)
            elif _is_cmp_comparer(a):
                comparer = a
        return self._q("AssumeRangePartition", key_selector=key_selector, descending=bool(is_descending),
                       separators=range_separators, comparer=comparer, dtype=self.dtype)

    def AssumeOrderBy(self, key_selector, is_descending=False, comparer=None):
        return self._q("AssumeOrderBy", key_selector=key_selector, descending=bool(is_descending),
                       comparer=comparer, dtype=self.dtype)

    # ----------------------------------------------------------------- Apply family
    def Apply(self, *args):
        """Apply(f) | Apply(other, f) | Apply([others], f): f sees whole inputs (merged to one
        partition) unless decorated @homomorphic, then it runs per partition."""
        others, func = _apply_args(args)
        srcs = [self._node] + [self._other(o) for o in others]
        multi = len(args) == 2 and isinstance(args[0], (list, tuple))
        return Query(self._ctx, QNode("Apply", srcs, dict(func=func, per_partition=False, multi=multi)))

    def ApplyPerPartition(self, *args, is_first_only: bool = False):
        others, func = _apply_args(args)
        srcs = [self._node] + [self._other(o) for o in others]
        multi = len(args) == 2 and isinstance(args[0], (list, tuple))
        return Query(self._ctx, QNode("Apply", srcs, dict(func=func, per_partition=True, multi=multi,
                                                          first_only=bool(is_first_only))))

    def ApplyWithPartitionIndex(self, func):
        return self._q("ApplyWithPartitionIndex", func=func)

    def SlidingWindow(self, func, window_size: int):
        if window_size < 2:
            raise DryadLinqException(ErrorCode.Unspecified, "SlidingWindow requires windowSize >= 2")  # SR.WindowSizeMustyBeGTOne
        return self._q("SlidingWindow", func=func, window_size=int(window_size))

    def DoWhile(self, body: Callable, cond: Callable, checkpoint: str | None = None) -> "Query":
        """Client-side loop (reference DryadLinqQueryable.cs:1280-1306): materialise body(before)
        each iteration; stop when cond(before, after) yields False.  ``checkpoint``: persist each
        iteration under that uri prefix so a rerun resumes after the last completed iteration."""
        return self._ctx._do_while(self, body, cond, checkpoint)

    def Fork(self, mapper, keys=None, per_record: bool = False):
        """Fork(mapper) -> MultiQuery with .First/.Second[/.Third]; Fork(keySel, keys) -> keyed."""
        if keys is not None:
            n = QNode("Fork", [self._node], dict(mapper=mapper, keys=list(keys), per_record=True))
            return KeyedMultiQuery(self._ctx, n, list(keys))
        n = QNode("Fork", [self._node], dict(mapper=mapper, keys=None, per_record=per_record))
        return MultiQuery(self._ctx, n)

    # ----------------------------------------------------------------- output / submission
    def ToStore(self, uri: str, delete_if_exists: bool = False, serializer=None, deserializer=None, dtype=None):
        return Query(self._ctx, QNode("ToStore", [self._node],
                                      dict(uri=str(uri), delete_if_exists=bool(delete_if_exists),
                                           serializer=serializer, deserializer=deserializer),
                                      dtype or self.dtype))

    def Submit(self):
        return self._ctx.Submit(self)

    def SubmitAndWait(self):
        return self._ctx.SubmitAndWait(self)


class MultiQuery:
    """IMultiQueryable<R1, R2[, R3]>: the outputs of one Fork."""

    def __init__(self, ctx, node: QNode):
        self._ctx, self._node = ctx, node

    def _port(self, i):
        return Query(self._ctx, QNode("ForkPort", [self._node], dict(port=i), port=i))

    @property
    def First(self):
        return self._port(0)

    @property
    def Second(self):
        return self._port(1)

    @property
    def Third(self):
        return self._port(2)

    def __getitem__(self, i):
        return self._port(i)


class KeyedMultiQuery(MultiQuery):
    """IKeyedMultiQueryable<T, K>: ``q[key]`` selects the records routed to ``key``."""

    def __init__(self, ctx, node, keys):
        super().__init__(ctx, node)
        self.keys = keys

    def __getitem__(self, key):
        try:
            i = self.keys.index(key)
        except ValueError:
            raise KeyError(key)
        return self._port(i)


def _aggregate_args(args):
    if len(args) == 1:
        return _NOSEED, args[0], None
    if len(args) == 2:
        return args[0], args[1], None
    if len(args) == 3:
        return args[0], args[1], args[2]
    raise TypeError("Aggregate(func) | Aggregate(seed, func) | Aggregate(seed, func, resultSelector)")


class _NoSeed:
    def __repr__(self):
        return "<no seed>"


_NOSEED = _NoSeed()


def _apply_args(args):
    if len(args) == 1:
        return [], args[0]
    if len(args) == 2:
        o, f = args
        if isinstance(o, (list, tuple)):
            return list(o), f
        return [o], f
    raise TypeError("Apply(f) | Apply(other, f) | Apply([others], f)")


def _check_separators(seps, comparer, descending):
    from .enumerable import compare_fn
    cmp = compare_fn(comparer)
    for a, b in zip(seps, seps[1:]):
        c = cmp(a, b)
        if (c > 0 and not descending) or (c < 0 and descending):
            raise DryadLinqException(ErrorCode.PartitionKeysAreNotConsistentlyOrdered,
                                     "range separators are not sorted in the partition order")


# snake_case aliases for every public operator
def _snake(name):
    out = []
    for i, c in enumerate(name):
        if c.isupper() and i and not name[i - 1].isupper():
            out.append("_")
        out.append(c.lower())
    return "".join(out)


for _cls in (Query,):
    for _name in [n for n in dir(_cls) if n[:1].isupper()]:
        _alias = _snake(_name)
        if not hasattr(_cls, _alias):
            setattr(_cls, _alias, getattr(_cls, _name))

"""LocalDebug oracle: LINQ-to-Objects semantics of every DryadLINQ operator over Python iterables.

This is the executable specification the distributed executors are tested against (the
reference's test suite runs each query on the cluster and in LocalDebug and compares).
It implements the standard LINQ operators with .NET ordering/laziness semantics plus the
DryadLINQ-only operators of ``DryadLinqEnumerable`` (reference LinqToDryad/DryadLinqEnumerable.cs:
HashPartition/RangePartition are identities (:42-126), Apply calls the function on the whole
sequence (:128-169), DoWhile loops body/cond (:171-186), SlidingWindow (:188-212),
ApplyWithPartitionIndex uses index 0 (:214-219), *AsQuery wrap scalars in one-element sequences).

It is also the object-level operator library that CPU vertices run on each partition.
"""
from __future__ import annotations

import functools
import heapq
import itertools
import math
from collections import OrderedDict, deque

from .errors import DryadLinqException, ErrorCode


class InvalidOperationException(DryadLinqException):
    """LINQ's InvalidOperationException for empty / ambiguous sequences, carrying the vertex
    runtime code the reference reports for the same condition (DryadLinqFaultCodes.cs:140-166)."""

    def __init__(self, msg, code=None):
        if code is None:
            m = msg.lower()
            code = (ErrorCode.SingleMoreThanOneElement if "more than one" in m else
                    ErrorCode.FirstNoElementsFirst if "matching" in m else ErrorCode.AggregateNoElements)
        super().__init__(code, msg)


# ---------------------------------------------------------------------------------------------
# comparers
def _has(o, name):
    return o is not None and hasattr(o, name)


class _EqKey:
    """Hashable wrapper applying a custom IEqualityComparer (Equals / GetHashCode)."""
    __slots__ = ("v", "c", "h")

    def __init__(self, v, c):
        self.v, self.c = v, c
        self.h = c.GetHashCode(v) if _has(c, "GetHashCode") else c.hash(v)

    def __hash__(self):
        return self.h

    def __eq__(self, o):
        return self.c.Equals(self.v, o.v) if _has(self.c, "Equals") else self.c.equals(self.v, o.v)


def eq_wrapper(comparer):
    """key -> hashable key honouring an optional equality comparer."""
    if comparer is None:
        return _hashable
    return lambda k: _EqKey(k, comparer)


def _hashable(k):
    if isinstance(k, list):
        return tuple(_hashable(x) for x in k)
    if isinstance(k, dict):
        return tuple(sorted(k.items()))
    return k


def _null_first_cmp(a, b):
    if a is None:
        return 0 if b is None else -1
    if b is None:
        return 1
    return -1 if a < b else (1 if b < a else 0)


def compare_fn(comparer=None):
    """Three-way compare honouring an optional IComparer (``Compare``) or cmp callable."""
    if comparer is None:
        return _null_first_cmp
    if _has(comparer, "Compare"):
        return comparer.Compare
    if callable(comparer):
        return comparer
    raise DryadLinqException(ErrorCode.ComparerMustBeSpecifiedOrKeyTypeMustBeIComparable, "bad comparer")


def sort_key(key_selector, comparer=None, descending=False):
    cmp = compare_fn(comparer)
    if descending:
        f = lambda a, b: -cmp(a, b)  # noqa: E731
    else:
        f = cmp
    K = functools.cmp_to_key(f)
    return lambda x: K(key_selector(x))


class LinqList(list):
    """A list with LINQ-to-Objects methods (what C# code gets on IEnumerable<T>)."""

    def Count(self, pred=None):
        return Count(self, pred)

    LongCount = Count

    def Sum(self, sel=None):
        return Sum(self, sel)

    def Min(self, sel=None):
        return Min(self, sel)

    def Max(self, sel=None):
        return Max(self, sel)

    def Average(self, sel=None):
        return Average(self, sel)

    def Any(self, pred=None):
        return Any(self, pred)

    def All(self, pred):
        return All(self, pred)

    def Contains(self, v):
        return Contains(self, v)

    def First(self, pred=None):
        return First(self, pred)

    def FirstOrDefault(self, pred=None):
        return FirstOrDefault(self, pred)

    def Last(self, pred=None):
        return Last(self, pred)

    def LastOrDefault(self, pred=None):
        return LastOrDefault(self, pred)

    def Single(self, pred=None):
        return Single(self, pred)

    def Aggregate(self, *args):
        if len(args) == 1:
            return Aggregate(self, _NO, args[0])
        return Aggregate(self, *args)

    def Select(self, f):
        return LinqList(Select(self, f, nparams_is2(f)))

    def Where(self, f):
        return LinqList(Where(self, f, nparams_is2(f)))

    def SelectMany(self, f, r=None):
        return LinqList(SelectMany(self, f, r))

    def OrderBy(self, k, comparer=None):
        return LinqList(OrderBy(self, k, comparer))

    def OrderByDescending(self, k, comparer=None):
        return LinqList(OrderBy(self, k, comparer, True))

    def Distinct(self, comparer=None):
        return LinqList(Distinct(self, comparer))

    def Take(self, n):
        return LinqList(self[:max(0, n)])

    def Skip(self, n):
        return LinqList(self[max(0, n):])

    def ToList(self):
        return list(self)

    ToArray = ToList


def nparams_is2(f):
    from .query import nparams
    return nparams(f) >= 2


class Grouping(LinqList):
    """IGrouping<K, T>: a list of elements with a ``Key``."""

    def __init__(self, key, elements=()):
        super().__init__(elements)
        self.Key = key

    def __repr__(self):
        return f"Grouping(Key={self.Key!r}, {list.__repr__(self)})"

    def __eq__(self, o):
        return isinstance(o, Grouping) and self.Key == o.Key and list.__eq__(self, o)

    def __hash__(self):
        return hash(self.Key)


# ---------------------------------------------------------------------------------------------
# standard operators
def Where(src, pred, indexed=False):
    if indexed:
        return (x for i, x in enumerate(src) if pred(x, i))
    return (x for x in src if pred(x))


def Select(src, sel, indexed=False):
    if indexed:
        return (sel(x, i) for i, x in enumerate(src))
    return (sel(x) for x in src)


def SelectMany(src, coll_sel, result_sel=None, indexed=False):
    for i, x in enumerate(src):
        coll = coll_sel(x, i) if indexed else coll_sel(x)
        for y in coll:
            yield result_sel(x, y) if result_sel is not None else y


def Take(src, n):
    return itertools.islice(src, max(0, n))


def Skip(src, n):
    return itertools.islice(src, max(0, n), None)


def TakeWhile(src, pred, indexed=False):
    for i, x in enumerate(src):
        if not (pred(x, i) if indexed else pred(x)):
            return
        yield x


def SkipWhile(src, pred, indexed=False):
    it = iter(src)
    i = 0
    for x in it:
        if not (pred(x, i) if indexed else pred(x)):
            yield x
            break
        i += 1
    yield from it


def OrderBy(src, key_sel, comparer=None, descending=False):
    return sorted(src, key=sort_key(key_sel, comparer, descending))   # stable


def OrderByDescending(src, key_sel, comparer=None):
    return OrderBy(src, key_sel, comparer, True)


def GroupBy(src, key_sel, elem_sel=None, result_sel=None, comparer=None):
    wrap = eq_wrapper(comparer)
    groups = OrderedDict()
    for x in src:
        k = key_sel(x)
        wk = wrap(k)
        g = groups.get(wk)
        if g is None:
            g = groups[wk] = Grouping(k)
        g.append(elem_sel(x) if elem_sel is not None else x)
    if result_sel is None:
        return list(groups.values())
    return [result_sel(g.Key, g) for g in groups.values()]


def Join(outer, inner, outer_key, inner_key, result_sel, comparer=None):
    wrap = eq_wrapper(comparer)
    table = {}
    for y in inner:
        k = inner_key(y)
        if k is None:
            continue
        table.setdefault(wrap(k), []).append(y)
    for x in outer:
        k = outer_key(x)
        if k is None:
            continue
        for y in table.get(wrap(k), ()):
            yield result_sel(x, y)


def GroupJoin(outer, inner, outer_key, inner_key, result_sel, comparer=None):
    wrap = eq_wrapper(comparer)
    table = {}
    for y in inner:
        k = inner_key(y)
        if k is None:
            continue
        table.setdefault(wrap(k), []).append(y)
    for x in outer:
        k = outer_key(x)
        # the group is an IEnumerable<TInner> in the reference: LINQ methods (g.Count(), g.Sum(...))
        yield result_sel(x, LinqList(table.get(wrap(k), ())) if k is not None else LinqList())


def Distinct(src, comparer=None):
    wrap = eq_wrapper(comparer)
    seen = set()
    for x in src:
        k = wrap(x)
        if k not in seen:
            seen.add(k)
            yield x


def Concat(a, b):
    return itertools.chain(a, b)


def Union(a, b, comparer=None):
    return Distinct(itertools.chain(a, b), comparer)


def Intersect(a, b, comparer=None):
    wrap = eq_wrapper(comparer)
    bs = {wrap(y) for y in b}
    for x in a:
        k = wrap(x)
        if k in bs:
            bs.discard(k)
            yield x


def Except(a, b, comparer=None):
    wrap = eq_wrapper(comparer)
    bs = {wrap(y) for y in b}
    for x in a:
        k = wrap(x)
        if k not in bs:
            bs.add(k)
            yield x


def Zip(a, b, result_sel):
    return (result_sel(x, y) for x, y in zip(a, b))


def Reverse(src):
    return list(src)[::-1]


# ---------------------------------------------------------------------------------------------
# aggregates
def _sel(src, sel):
    return src if sel is None else (sel(x) for x in src)


def Count(src, pred=None):
    return sum(1 for x in src if pred is None or pred(x))


LongCount = Count


def Any(src, pred=None):
    return any(True for x in src if pred is None or pred(x))


def All(src, pred):
    return all(pred(x) for x in src)


def Contains(src, value, comparer=None):
    if comparer is None:
        return any(x == value for x in src)
    eq = comparer.Equals if _has(comparer, "Equals") else comparer.equals
    return any(eq(x, value) for x in src)


def SequenceEqual(a, b, comparer=None):
    eq = (lambda x, y: x == y) if comparer is None else (
        comparer.Equals if _has(comparer, "Equals") else comparer.equals)
    sentinel = object()
    for x, y in itertools.zip_longest(a, b, fillvalue=sentinel):
        if x is sentinel or y is sentinel or not eq(x, y):
            return False
    return True


_NO = object()


def First(src, pred=None, default=_NO):
    for x in src:
        if pred is None or pred(x):
            return x
    if default is _NO:
        raise InvalidOperationException("Sequence contains no (matching) elements")
    return default


def FirstOrDefault(src, pred=None):
    return First(src, pred, None)


def Last(src, pred=None, default=_NO):
    found, last = False, None
    for x in src:
        if pred is None or pred(x):
            found, last = True, x
    if not found:
        if default is _NO:
            raise InvalidOperationException("Sequence contains no (matching) elements")
        return default
    return last


def LastOrDefault(src, pred=None):
    return Last(src, pred, None)


def Single(src, pred=None, default=_NO):
    found, val = False, None
    for x in src:
        if pred is None or pred(x):
            if found:
                raise InvalidOperationException("Sequence contains more than one (matching) element")
            found, val = True, x
    if not found:
        if default is _NO:
            raise InvalidOperationException("Sequence contains no (matching) elements")
        return default
    return val


def SingleOrDefault(src, pred=None):
    return Single(src, pred, None)


def Sum(src, sel=None):
    tot = 0
    for v in _sel(src, sel):
        if v is not None:
            tot = tot + v
    return tot


def Min(src, sel=None, comparer=None):
    best, found = None, False
    cmp = compare_fn(comparer)
    for v in _sel(src, sel):
        if v is None:
            continue
        if not found or cmp(v, best) < 0:
            best, found = v, True
    if not found:
        raise InvalidOperationException("Sequence contains no elements")
    return best


def Max(src, sel=None, comparer=None):
    best, found = None, False
    cmp = compare_fn(comparer)
    for v in _sel(src, sel):
        if v is None:
            continue
        if not found or cmp(v, best) > 0:
            best, found = v, True
    if not found:
        raise InvalidOperationException("Sequence contains no elements")
    return best


def Average(src, sel=None):
    tot, n = 0, 0
    for v in _sel(src, sel):
        if v is None:
            continue
        tot += v
        n += 1
    if n == 0:
        raise InvalidOperationException("Sequence contains no elements")
    return tot / n


def Aggregate(src, seed=_NO, func=None, result_sel=None):
    it = iter(src)
    if seed is _NO:
        try:
            acc = next(it)
        except StopIteration:
            raise InvalidOperationException("Sequence contains no elements")
    else:
        acc = seed
    for x in it:
        acc = func(acc, x)
    return result_sel(acc) if result_sel is not None else acc


# ---------------------------------------------------------------------------------------------
# DryadLINQ extensions (LocalDebug semantics)
def HashPartition(src, key_sel, comparer=None, count=None, result_sel=None):
    return src if result_sel is None else (result_sel(x) for x in src)


def RangePartition(src, key_sel, *args, **kw):
    return src


def AssumeHashPartition(src, *a, **k):
    return src


def AssumeRangePartition(src, *a, **k):
    return src


def AssumeOrderBy(src, *a, **k):
    return src


def Apply(src, func, *others):
    return func(src, *others)


def ApplyPerPartition(src, func, *others):
    return func(src, *others)


def ApplyWithPartitionIndex(src, func):
    return func(src, 0)


def SlidingWindow(src, func, window_size):
    if window_size < 2:
        raise DryadLinqException(ErrorCode.Unspecified,  # SR.WindowSizeMustyBeGTOne (message-only ctor)
                                 "windowSize must be at least 2")
    win = deque(maxlen=window_size)
    for x in src:
        win.append(x)
        if len(win) == window_size:
            yield func(list(win))


def Fork(src, mapper, keys=None):
    """Fork: one pass, several outputs.  ``mapper`` maps the whole sequence to ForkTuples
    (2/3-way) or, with ``keys``, routes each record to the output whose key matches."""
    from .types import ForkTuple
    src = list(src)
    if keys is not None:
        outs = [[] for _ in keys]
        idx = {k: i for i, k in enumerate(keys)}
        for x in src:
            i = idx.get(mapper(x))
            if i is not None:
                outs[i].append(x)
        return outs
    outs = None
    for t in mapper(src):
        if not isinstance(t, ForkTuple):
            raise DryadLinqException(ErrorCode.FailureInUserApplyFunction, "Fork mapper must yield ForkTuple values")
        vals = (t.First, t.Second, t.Third)
        if outs is None:
            outs = [[], [], []]
        for i, v in enumerate(vals):
            if v.HasValue:
                outs[i].append(v.Value)
    return outs or [[], [], []]


def Offsets(counts):
    """Per-partition start offsets from counts (reference DryadLinqEnumerable.Offsets)."""
    out, acc = [], 0
    for c in counts:
        out.append(acc)
        acc += c
    return out


def MergeSort(runs, key_sel, comparer=None, descending=False):
    """k-way merge of sorted runs (reference DryadLinqVertex.MergeSort :319-423)."""
    k = sort_key(key_sel, comparer, descending)
    return heapq.merge(*runs, key=k)


def isclose(a, b):
    if isinstance(a, float) or isinstance(b, float):
        return math.isclose(a, b, rel_tol=1e-9, abs_tol=1e-12)
    return a == b

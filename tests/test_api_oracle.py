"""Operator coverage: every query runs distributed (CPU vertex hosts, 3 partitions) and in
LocalDebug, results compared (reference BasicAPITests / GroupByReduceTests / MiscBugFixTests
scenarios)."""
import dataclasses

import pytest

import dryad_amd as D
from dryad_amd.errors import DryadLinqException, ErrorCode
from helpers import both, cluster_ctx, local_ctx

N = list(range(200))


def test_where_select():
    both(lambda c: c.FromEnumerable(N).Where(lambda x: x % 3 == 0).Select(lambda x: x * 2 + 1))


def test_select_preserves_order():
    both(lambda c: c.FromEnumerable(N).Select(lambda x: x * 7 % 101), ordered=True)


def test_indexed_select_where_selectmany():
    both(lambda c: c.FromEnumerable(N).Select(lambda x, i: (x, i)), ordered=True)
    both(lambda c: c.FromEnumerable(N).Where(lambda x, i: i % 5 == 0), ordered=True)
    both(lambda c: c.FromEnumerable(N[:30]).SelectMany(lambda x, i: [i] * (x % 3)), ordered=True)
    both(lambda c: c.FromEnumerable(N).LongSelect(lambda x, i: x + i), ordered=True)


def test_selectmany_result_selector():
    both(lambda c: c.FromEnumerable(["a b", "c", "d e f"]).SelectMany(lambda s: s.split(), lambda s, w: (s, w)))


def test_take_skip_while():
    both(lambda c: c.FromEnumerable(N).Take(17), ordered=True)
    both(lambda c: c.FromEnumerable(N).Skip(190), ordered=True)
    both(lambda c: c.FromEnumerable(N).TakeWhile(lambda x: x < 50), ordered=True)
    both(lambda c: c.FromEnumerable(N).SkipWhile(lambda x: x < 150), ordered=True)
    both(lambda c: c.FromEnumerable(N).TakeWhile(lambda x, i: i < 10), ordered=True)


def test_orderby_and_descending():
    data = [(i * 37) % 211 for i in range(300)]
    both(lambda c: c.FromEnumerable(data).OrderBy(lambda x: x), ordered=True)
    both(lambda c: c.FromEnumerable(data).OrderByDescending(lambda x: x % 13), ordered=False)
    r = list(cluster_ctx().FromEnumerable(data).OrderByDescending(lambda x: x))
    assert r == sorted(data, reverse=True)


def test_orderby_is_stable_within_equal_keys():
    data = [(i % 4, i) for i in range(100)]
    r = list(cluster_ctx().FromEnumerable(data).OrderBy(lambda t: t[0]))
    assert [t[0] for t in r] == sorted(t[0] for t in data)


def test_thenby_not_supported():
    with pytest.raises(DryadLinqException) as e:
        local_ctx().FromEnumerable(N).OrderBy(lambda x: x).ThenBy(lambda x: x)
    assert e.value.ErrorCode == ErrorCode.OperatorNotSupported


def test_groupby_variants():
    words = ["apple", "bob", "cat", "apple", "dog", "cat", "apple", "eel"] * 7
    both(lambda c: c.FromEnumerable(words).GroupBy(lambda w: w))
    both(lambda c: c.FromEnumerable(words).GroupBy(lambda w: w[0], lambda w: len(w)))
    both(lambda c: c.FromEnumerable(words).GroupBy(lambda w: w, lambda k, g: (k, g.Count())))
    both(lambda c: c.FromEnumerable(words).GroupBy(lambda w: len(w), lambda w: w.upper(), lambda k, g: (k, sorted(g))))


def test_groupby_decomposable_aggregates():
    data = [(i % 7, float(i)) for i in range(500)]
    both(lambda c: c.FromEnumerable(data).GroupBy(
        lambda t: t[0], lambda k, g: (k, g.Count(), g.Sum(lambda t: t[1]), g.Min(lambda t: t[1]),
                                      g.Max(lambda t: t[1]), g.Average(lambda t: t[1]))))
    both(lambda c: c.FromEnumerable(data).GroupBy(
        lambda t: t[0], lambda k, g: {"k": k, "ratio": g.Sum(lambda t: t[1]) / g.Count(),
                                      "any": g.Any(lambda t: t[1] > 400), "all": g.All(lambda t: t[1] >= 0)}))


def test_groupby_decomposition_is_used():
    c = cluster_ctx()
    q = c.FromEnumerable(N).GroupBy(lambda x: x % 3, lambda k, g: (k, g.Count()))
    assert "group_partial" in c.Explain(q)
    q2 = c.FromEnumerable(N).GroupBy(lambda x: x % 3, lambda k, g: (k, len(g)))
    assert "group_partial" not in c.Explain(q2)
    both(lambda c: c.FromEnumerable(N).GroupBy(lambda x: x % 3, lambda k, g: (k, len(g))))


class SumSquares(D.IDecomposable):
    def Seed(self, x):
        return x * x

    def Accumulate(self, a, x):
        return a + x * x

    def RecursiveAccumulate(self, a, b):
        return a + b

    def FinalReduce(self, a):
        return a


@D.decomposable(SumSquares)
def sum_squares(g):
    return sum(x * x for x in g)


def test_user_decomposable():
    both(lambda c: c.FromEnumerable(N).GroupBy(lambda x: x % 5, lambda k, g: (k, sum_squares(g))))
    assert "group_partial" in cluster_ctx().Explain(
        cluster_ctx().FromEnumerable(N).GroupBy(lambda x: x % 5, lambda k, g: (k, sum_squares(g))))


class CaseInsensitive:
    def Equals(self, a, b):
        return a.lower() == b.lower()

    def GetHashCode(self, a):
        return sum(ord(ch) for ch in a.lower())


def test_groupby_with_comparer():
    words = ["Ab", "aB", "cd", "CD", "x"] * 5
    r = both(lambda c: c.FromEnumerable(words).GroupBy(lambda w: w, lambda k, g: (k.lower(), g.Count()),
                                                       comparer=CaseInsensitive()))
    assert sorted(r) == [("ab", 10), ("cd", 10), ("x", 5)]


def test_join_and_groupjoin():
    cust = [(i, f"c{i}") for i in range(40)]
    orders = [(i % 50, i * 1.5) for i in range(120)]
    both(lambda c: c.FromEnumerable(cust).Join(c.FromEnumerable(orders), lambda a: a[0], lambda o: o[0],
                                               lambda a, o: (a[1], o[1])))
    both(lambda c: c.FromEnumerable(cust).GroupJoin(c.FromEnumerable(orders), lambda a: a[0], lambda o: o[0],
                                                    lambda a, os: (a[1], len(os))))


def test_set_operations():
    a = [i % 30 for i in range(100)]
    b = [i % 17 + 10 for i in range(50)]
    both(lambda c: c.FromEnumerable(a).Distinct())
    both(lambda c: c.FromEnumerable(a).Union(c.FromEnumerable(b)))
    both(lambda c: c.FromEnumerable(a).Intersect(c.FromEnumerable(b)))
    both(lambda c: c.FromEnumerable(a).Except(c.FromEnumerable(b)))
    both(lambda c: c.FromEnumerable(a).Concat(c.FromEnumerable(b)), ordered=True)


def test_zip_reverse():
    both(lambda c: c.FromEnumerable(N).Zip(c.FromEnumerable(N[::-1]), lambda x, y: x - y), ordered=True)
    both(lambda c: c.FromEnumerable(N).Reverse(), ordered=True)


def test_scalar_aggregates():
    for f in [lambda q: q.Count(), lambda q: q.Count(lambda x: x > 10), lambda q: q.LongCount(),
              lambda q: q.Sum(), lambda q: q.Sum(lambda x: x * 0.5), lambda q: q.Min(), lambda q: q.Max(),
              lambda q: q.Average(), lambda q: q.Any(), lambda q: q.Any(lambda x: x > 1000),
              lambda q: q.All(lambda x: x >= 0), lambda q: q.Contains(77), lambda q: q.First(),
              lambda q: q.First(lambda x: x > 100), lambda q: q.FirstOrDefault(lambda x: x > 1000),
              lambda q: q.Last(), lambda q: q.LastOrDefault(lambda x: x < 0), lambda q: q.Single(lambda x: x == 5),
              lambda q: q.SingleOrDefault(lambda x: x == -5), lambda q: q.Aggregate(lambda a, b: a + b),
              lambda q: q.Aggregate(10, lambda a, b: a + b, lambda r: r * 2)]:
        both(lambda c: f(c.FromEnumerable(N)))


def test_scalar_errors():
    with pytest.raises(Exception):
        cluster_ctx().FromEnumerable([]).First()
    with pytest.raises(Exception):
        cluster_ctx().FromEnumerable(N).Single()


def test_as_query_variants():
    both(lambda c: c.FromEnumerable(N).CountAsQuery())
    both(lambda c: c.FromEnumerable(N).SumAsQuery(lambda x: x))
    both(lambda c: c.FromEnumerable(N).AnyAsQuery(lambda x: x > 5))
    both(lambda c: c.FromEnumerable(N).MaxAsQuery())
    both(lambda c: c.FromEnumerable(N).SequenceEqualAsQuery(c.FromEnumerable(N)))


def test_sequence_equal():
    both(lambda c: c.FromEnumerable(N).SequenceEqual(c.FromEnumerable(N)))
    both(lambda c: c.FromEnumerable(N).SequenceEqual(c.FromEnumerable(N[:-1])))


def test_hash_partition_overloads():
    both(lambda c: c.FromEnumerable(N).HashPartition(lambda x: x % 10))
    both(lambda c: c.FromEnumerable(N).HashPartition(lambda x: x % 10, 5))
    both(lambda c: c.FromEnumerable(N).HashPartition(lambda x: x % 10, lambda x: -x))
    c = cluster_ctx()
    q = c.FromEnumerable(N).HashPartition(lambda x: x % 10, 4).ApplyWithPartitionIndex(
        lambda s, i: [(i, x % 10) for x in s])
    parts = {}
    for i, k in q:
        parts.setdefault(k, set()).add(i)
    assert all(len(v) == 1 for v in parts.values())       # equal keys -> one partition


@dataclasses.dataclass(frozen=True)
class Point:
    x: int
    y: str


def test_user_types_in_query():
    pts = [Point(i % 9, f"p{i}") for i in range(60)]
    both(lambda c: c.FromEnumerable(pts).Where(lambda p: p.x > 2).GroupBy(lambda p: p.x, lambda k, g: Point(k, str(g.Count()))))
    both(lambda c: c.FromEnumerable(pts).Select(lambda p: {"x": p.x}["x"]).Distinct())


def test_concat_keeps_partition_order():
    both(lambda c: c.FromEnumerable([1, 2, 3]).Concat(c.FromEnumerable([4, 5])).Select(lambda x: x * 10), ordered=True)


def test_empty_inputs():
    both(lambda c: c.FromEnumerable([]).Where(lambda x: True))
    both(lambda c: c.FromEnumerable([]).GroupBy(lambda x: x))
    both(lambda c: c.FromEnumerable([]).Count())
    both(lambda c: c.FromEnumerable([]).OrderBy(lambda x: x), ordered=True)


def test_shared_subquery_tee():
    def build(c):
        base = c.FromEnumerable(N).Select(lambda x: x % 11)
        return base.Where(lambda x: x > 5).Concat(base.Where(lambda x: x <= 5))
    both(build)


def test_sliding_window():
    both(lambda c: c.FromEnumerable(N[:20]).SlidingWindow(lambda w: sum(w), 3), ordered=True)


def test_aggregation_tree_for_wide_aggregates():
    import dryad_amd as D
    c = D.DryadLinqContext(2)
    c.PartitionCount = 40
    c.AggregationTreeMaxInputs = 6
    c.AggregationTreeGroup = 4
    data = list(range(1, 2001))
    q = c.FromEnumerable(data)
    plan = c.Explain(q.Select(lambda x: x * 2).Where(lambda x: x % 3 == 0))
    assert plan
    assert q.Sum() == sum(data)
    assert q.Count() == len(data)
    assert q.Min() == 1 and q.Max() == 2000
    assert abs(q.Average() - sum(data) / len(data)) < 1e-9
    assert q.First(lambda x: x > 1500) == 1501 and q.Last(lambda x: x < 10) == 9
    assert q.Any(lambda x: x == 1999) and not q.All(lambda x: x < 1000)
    from dryad_amd.compiler.planner import compile_queries
    p = compile_queries(c, [q.SumAsQuery()])
    assert any("Combine" in s.name for s in p.stages)

"""Planner strategies of the reference's QueryGen that elide shuffles and sorts (CPU):
OrderedGroupBy on sorted input (DryadLinqQueryGen.cs:2098-2100), merge join when one side is
ordered (:1574-1597) with range co-partitioning (:1487-1512), ordered Distinct / set operations
(:1862-1880), and the Phase-3 removal of useless Merge vertices (:474-500).  Each plan is
checked through Explain, each result against the LocalDebug oracle on the process executor
(and the SPMD executor on one CPU rank)."""
import pytest

import dryad_amd as D
from dryad_amd.compiler.planner import compile_queries

DATA = [(i * 7919) % 5003 for i in range(6000)]
PAIRS = [(i % 61, i) for i in range(4000)]


def _ctx(kind):
    if kind == "local":
        c = D.DryadLinqContext(1)
        c.LocalDebug = True
        return c
    if kind == "proc":
        c = D.DryadLinqContext(2)
        c.PartitionCount = 3
        return c
    c = D.DryadLinqContext(platform="gpu")
    c.PartitionCount = 3
    return c


def _ops(q, ctx):
    p = compile_queries(ctx, [q.ToStore("mem://planner_probe", delete_if_exists=True)])
    return p, [o["op"] for s in p.stages for o in s.ops]


def _check(build, ordered=False):
    exp = list(build(_ctx("local")))
    for kind in ("proc", "spmd"):
        got = list(build(_ctx(kind)))
        if ordered:
            assert got == exp, kind
        else:
            assert sorted(got, key=repr) == sorted(exp, key=repr), kind


def test_orderby_then_groupby_is_ordered_group_by_without_second_shuffle():
    def q(c):
        return c.FromEnumerable(PAIRS).OrderBy(lambda t: t[0]).GroupBy(
            lambda t: t[0], lambda k, g: (k, g.Count(), g.Sum(lambda t: t[1])))
    plan, ops = _ops(q(_ctx("proc")), _ctx("proc"))
    assert "ordered_group_by" in ops and "hash_partition" not in ops and "group_partial" not in ops
    assert ops.count("range_partition") == 1
    assert "no sort" in plan.explain()
    _check(q)


def test_merge_join_with_one_ordered_side_co_range_partitions_the_other():
    def q(c):
        outer = c.FromEnumerable(PAIRS).OrderBy(lambda t: t[0])
        inner = c.FromEnumerable([(k, k * 10) for k in range(0, 61, 2)])
        return outer.Join(inner, lambda t: t[0], lambda u: u[0], lambda t, u: (t[1], u[1]))
    plan, ops = _ops(q(_ctx("proc")), _ctx("proc"))
    assert "merge_join" in ops and "hash_join" not in ops and "hash_partition" not in ops
    assert ops.count("range_partition") == 2 and ops.count("sample") == 1     # the inner reuses the separators
    ex = plan.explain()
    assert "inner sorted per partition" in ex and "separators of stage" in ex
    _check(q)


def test_distinct_of_sorted_input_drops_adjacent_duplicates():
    def q(c):
        return c.FromEnumerable([x % 300 for x in DATA]).OrderBy(lambda x: x).Distinct()
    plan, ops = _ops(q(_ctx("proc")), _ctx("proc"))
    assert "ordered_distinct" in ops and "hash_partition" not in ops
    _check(q)


def test_set_operations_on_sorted_inputs_merge():
    def q(c, kind):
        a = c.FromEnumerable([x % 400 for x in DATA]).OrderBy(lambda x: x)
        b = c.FromEnumerable([x % 250 for x in DATA[:3000]])
        return getattr(a, kind)(b)
    for kind in ("Union", "Intersect", "Except"):
        plan, ops = _ops(q(_ctx("proc"), kind), _ctx("proc"))
        assert "ordered_" + kind.lower() in ops, (kind, ops)
        assert "hash_partition" not in ops
        _check(lambda c, k=kind: q(c, k))


def test_useless_merge_vertices_removed():
    def q(c):
        return c.FromEnumerable(PAIRS).Join(c.FromEnumerable(PAIRS[:500]), lambda t: t[0], lambda u: u[0],
                                            lambda t, u: t[1] - u[1])
    plan, ops = _ops(q(_ctx("proc")), _ctx("proc"))
    join = next(s for s in plan.stages if any(o["op"] == "hash_join" for o in s.ops))
    assert [i.kind for i in join.inputs] == ["cross", "cross"] and join.gang
    assert not any(s.ops == [{"op": "identity", "explain": "merge"}] for s in plan.stages)
    assert "vertex elided" in plan.explain()
    _check(q)


@pytest.mark.parametrize("desc", [False, True])
def test_merge_join_descending_order(desc):
    def q(c):
        outer = c.FromEnumerable(PAIRS[:1500])
        outer = outer.OrderByDescending(lambda t: t[0]) if desc else outer.OrderBy(lambda t: t[0])
        return outer.Join(c.FromEnumerable([(k, -k) for k in range(0, 61, 3)]), lambda t: t[0], lambda u: u[0],
                          lambda t, u: (t[1], u[1]))
    _check(q)


def test_expensive_associative_aggregate_gets_full_aggregator():
    class AddAssoc:
        def Seed(self):
            return 0

        def RecursiveAccumulate(self, a, b):
            return a + b

    @D.resource(is_expensive=True)
    @D.associative(AddAssoc)
    def add(a, x):
        return a + x
    c = _ctx("proc")
    p = compile_queries(c, [c.FromEnumerable(DATA).AggregateAsQuery(0, add).ToStore("mem://fa", delete_if_exists=True)])
    final = next(s for s in p.stages if any(o["op"] == "agg_final" for o in s.ops))
    assert final.dynamic_manager == "FullAggregator"
    assert "<Type>FullAggregator</Type>" in p.to_xml()
    assert all(list(c2.FromEnumerable(DATA).Aggregate(0, add) for c2 in [_ctx(k)])[0] == sum(DATA)
               for k in ("local", "proc", "spmd"))


def test_exchange_one_rank_plans_the_range_shuffle():
    """ExchangeOneRank (the one-rank RCCL rehearsal, bench.py --rccl-one-rank): a one-partition
    OrderBy is planned as Sample -> Separators -> RangePartition -(cross)-> Merge+sort, and the
    query still gives the oracle's order on one CPU rank."""
    c = D.DryadLinqContext(platform="gpu")
    c.PartitionCount = 1
    c.ExchangeOneRank = True
    q = c.FromEnumerable(DATA).OrderBy(lambda x: x)
    p, ops = _ops(q, c)
    assert {"sample", "separators", "range_partition", "sort"} <= set(ops), ops
    assert list(q) == sorted(DATA)
    c1 = D.DryadLinqContext(platform="gpu")
    c1.PartitionCount = 1
    _, ops1 = _ops(c1.FromEnumerable(DATA).OrderBy(lambda x: x), c1)
    assert "range_partition" not in ops1, ops1

"""Named parity tests for the reference's regression suites (DryadLinqTests/MiscBugFixTests.cs,
BasicAPITests.cs, TypesInQueryTests.cs).  One test per reference method whose behaviour is not
already pinned elsewhere; each uses the reference's oracle pattern (the query runs on the
LocalDebug evaluator and on the multi-process executor and the results must agree) or checks the
error the reference expects.  Data: DataGenerator.GetSimpleFileSets-shaped inputs (Utils.cs:59-160:
small int sets over 3 partitions), built in the test."""
import dataclasses
import os
from typing import Optional

import pytest

import dryad_amd as D
from dryad_amd.errors import DryadLinqException, ErrorCode
from helpers import both, canon, cluster_ctx, local_ctx

SIMPLE = list(range(1, 41))               # GetSimpleFileSets: 1..40 over 3 parts
GBR = [(i * 37) % 101 for i in range(200)]  # GetGroupByReduceDataSet-shaped ints


def _simple(c):
    """Hash-partitioned input: record order depends on the partitioning, so the indexed-operator
    tests read the plain (source-ordered) input instead, as the reference's file sets do."""
    return c.FromEnumerable(SIMPLE).HashPartition(lambda x: x, 3)


# ------------------------------------------------------------------ MiscBugFixTests.cs
def test_Bug12584_HashPartitionOutputCount(tmp_path):
    c = cluster_ctx()
    uri = f"partfile://{tmp_path}/hp"
    c.FromEnumerable(SIMPLE).HashPartition(lambda x: x, 5).ToStore(uri, delete_if_exists=True).SubmitAndWait()
    lines = open(f"{tmp_path}/hp").read().splitlines()
    assert int(lines[1]) == 5                      # one output partition per hash bucket
    assert sorted(c.FromStore(uri)) == SIMPLE


def test_Bug13108_SequenceEqual():
    assert both(lambda c: _simple(c).Select(lambda x: x).SequenceEqual(_simple(c).Select(lambda x: x))) is True


def test_Bug13529_and_Bug13593_IndexedOperatorCompilation():
    both(lambda c: c.FromEnumerable(SIMPLE).Select(lambda x, i: x).LongSelect(lambda x, i: x + i).Where(lambda x, i: i % 2 == 0)
         .LongWhere(lambda x, i: i < 100).SelectMany(lambda x, i: [x, i]), ordered=True)


def test_Bug13130_ReverseOperator():
    both(lambda c: c.FromEnumerable(SIMPLE).Reverse(), ordered=True)
    both(lambda c: _simple(c).OrderBy(lambda x: x).Reverse(), ordered=True)


def test_Bug13736_IndexedTakeWhile():
    both(lambda c: c.FromEnumerable(SIMPLE).TakeWhile(lambda x, i: i < 17), ordered=True)


@pytest.mark.parametrize("count", [0, -1])
def test_Bug13534_HashPartitionNegIndexIsError(count):
    for c in (local_ctx(), cluster_ctx()):
        with pytest.raises(ValueError):
            _simple(c).HashPartition(lambda x: x, count)
        with pytest.raises(ValueError):
            _simple(c).RangePartition(lambda x: x, count)


def test_Bug13474_and_Bug13483_FromStoreOnBadFileSet(tmp_path):
    for c in (local_ctx(), cluster_ctx()):
        with pytest.raises(DryadLinqException):
            c.FromStore(f"partfile://{tmp_path}/does_not_exist")


def test_Bug13637_EmptyFilesInFilesets(tmp_path):
    c = cluster_ctx()
    uri = f"partfile://{tmp_path}/sparse"
    # two of the five partitions receive no records: their part files are empty
    c.FromEnumerable([3, 8, 13, 18]).HashPartition(lambda x: x % 5 // 3, 5).ToStore(uri, delete_if_exists=True) \
        .SubmitAndWait()
    assert sorted(c.FromStore(uri)) == [3, 8, 13, 18]
    assert sorted(local_ctx().FromStore(uri)) == [3, 8, 13, 18]


def test_Bug13637_LocalDebugProducingZeroRecords(tmp_path):
    for c in (local_ctx(), cluster_ctx()):
        uri = f"partfile://{tmp_path}/zero_{id(c)}"
        c.FromEnumerable(SIMPLE).Where(lambda x: x > 1000).ToStore(uri, delete_if_exists=True).SubmitAndWait()
        assert list(c.FromStore(uri)) == []


def test_Bug13970_MismatchedDataTypes():
    r = both(lambda c: list(c.FromEnumerable(GBR).AverageAsQuery())[0])
    assert r == pytest.approx(sum(GBR) / len(GBR))


def test_Bug14010_AlreadyDisposedContext():
    ctx = D.DryadLinqContext(2)
    ctx.Dispose()
    with pytest.raises(DryadLinqException) as e:
        ctx.FromEnumerable(SIMPLE).Select(lambda x: x).First()
    assert e.value.ErrorCode == ErrorCode.ContextDisposed
    ctx = D.DryadLinqContext(2)
    q = ctx.FromEnumerable(SIMPLE)
    ctx.Dispose()
    with pytest.raises(DryadLinqException):
        q.Select(lambda x: x).First()
    with pytest.raises(DryadLinqException):
        q.Select(lambda x: x).Submit()


def test_Bug14189_OrderPreservation():
    both(lambda c: _simple(c).OrderBy(lambda x: -x).Select(lambda x: x * 2).Where(lambda x: x % 3 != 0), ordered=True)


def test_Bug14190_MergeJoin_DecreasingOrder():
    both(lambda c: _simple(c).OrderByDescending(lambda x: x).Join(
        c.FromEnumerable(SIMPLE).OrderByDescending(lambda x: x), lambda x: x, lambda y: y, lambda x, y: x + y))


def test_Bug14192_MultiApplySubExpressionReuse():
    r = both(lambda c: _simple(c).Apply([_simple(c), _simple(c)], lambda sources: [1, 2, 3]))
    assert sorted(r) == [1, 2, 3]


def test_Bug14870_LongIndexTakeWhile():
    both(lambda c: c.FromEnumerable(SIMPLE).LongTakeWhile(lambda x, i: i < 23), ordered=True)


def test_Bug15159_NotOperatorForNullableBool():
    data: list = [True, None, False, True, None]
    both(lambda c: c.FromEnumerable(data).Where(lambda b: not (b is True)).Select(lambda b: b is None))


def test_Bug15570_GetHashCodeAndEqualsForNullableFieldsOfAnonymousTypes():
    data = [(i % 3, None if i % 2 else i % 4) for i in range(60)]
    r = both(lambda c: c.FromEnumerable(data).GroupBy(lambda t: (t[0], t[1]), lambda k, g: (k, g.Count())))
    assert sum(n for _, n in r) == 60 and len(r) == len(set(data))
    both(lambda c: c.FromEnumerable(data).Distinct())


# ------------------------------------------------------------------ BasicAPITests.cs
def test_ToStoreThrowsForNonQuery():
    with pytest.raises(DryadLinqException) as e:
        cluster_ctx().Submit([1, 2, 3])
    assert e.value.ErrorCode == ErrorCode.MustStartFromContext


def test_SubmitNonToStoreTerminated():
    c = cluster_ctx()
    q2 = _simple(c).Select(lambda x: 100 + x).Where(lambda x: True)
    q2.SubmitAndWait()
    assert sorted(q2) == [100 + x for x in SIMPLE]


def test_MaterializeNonToStoreTerminated():
    c = cluster_ctx()
    q = _simple(c).Select(lambda x: 100 + x)
    c.Submit(q).Wait()
    assert canon(q) == canon(local_ctx().FromEnumerable(SIMPLE).Select(lambda x: 100 + x))


def test_MaterializeMentionsSameQueryTwice(tmp_path):
    c = cluster_ctx()
    q = _simple(c).Select(lambda x: x + 1).ToStore(f"partfile://{tmp_path}/twice", delete_if_exists=True)
    info = c.SubmitAndWait(q, q)
    assert len(info.JobIds) == 1
    assert sorted(c.FromStore(f"partfile://{tmp_path}/twice")) == [x + 1 for x in SIMPLE]


def test_Bug11781_CountandFirstOrDefault():
    assert both(lambda c: _simple(c).Count()) == len(SIMPLE)
    assert both(lambda c: _simple(c).Where(lambda x: x > 10**6).FirstOrDefault()) is None


def test_Bug11782_Aggregate():
    assert both(lambda c: _simple(c).Aggregate(lambda a, x: a + x)) == sum(SIMPLE)
    assert both(lambda c: _simple(c).Aggregate(7, lambda a, x: a + 2 * x, lambda a: a * 10)) == (7 + 2 * sum(SIMPLE)) * 10


def test_Bug11638_LongMethods():
    both(lambda c: c.FromEnumerable(SIMPLE).LongWhere(lambda x, i: i % 3 == 1).LongSelect(lambda x, i: (x, i)).Select(lambda t: t[0]))
    both(lambda c: c.FromEnumerable(SIMPLE).LongSelectMany(lambda x, i: [x] * (i % 2)))
    assert both(lambda c: _simple(c).LongCount(lambda x: x % 2 == 0)) == 20


def test_Bug15068_ConfigResourcesAPI():
    c = D.DryadLinqContext(2)
    c.ResourcesToAdd.clear()
    c.ResourcesToRemove.clear()
    c.ResourcesToAdd.append("abc")
    c.ResourcesToRemove.extend(["def", "ghi"])
    assert c.ResourcesToAdd[0] == "abc" and len(c.ResourcesToAdd) == 1
    assert c.ResourcesToRemove[1] == "ghi" and len(c.ResourcesToRemove) == 2


def test_Bug14449_ContextShouldExposeVersionIDs():
    c = D.DryadLinqContext(2)
    assert c.ClientVersion() and c.ServerVersion()


def test_Bug_16341_SubmitThrowsForDifferentContexts():
    c1, c2 = D.DryadLinqContext(2), D.DryadLinqContext(2)
    for submit in (c1.Submit, c1.SubmitAndWait):
        with pytest.raises(DryadLinqException) as e:
            submit(_simple(c1), _simple(c2))
        assert e.value.ErrorCode == ErrorCode.MustStartFromContext


# ------------------------------------------------------------------ TypesInQueryTests.cs
@dataclasses.dataclass(frozen=True)
class Base:
    a: int


@dataclasses.dataclass(frozen=True)
class Derived(Base):
    b: Optional[str] = None


def test_NonSealedTypeRecords_and_DerivedTypeRecords():
    data = [Base(i) for i in range(20)] + [Derived(i, str(i)) for i in range(20)]
    both(lambda c: c.FromEnumerable(data).Where(lambda r: r.a % 2 == 0).Select(lambda r: (type(r).__name__, r.a)))
    both(lambda c: c.FromEnumerable(data).GroupBy(lambda r: type(r).__name__, lambda k, g: (k, g.Count())))


def test_ObjectRecords():
    data = [1, "two", 3.0, (4, "four"), None, Base(6)]
    both(lambda c: c.FromEnumerable(data).Select(lambda x: repr(x)))


def test_GroupByWithAnonymousTypes_Pipeline_and_Nested():
    data = [(i % 4, i % 3, i) for i in range(90)]
    both(lambda c: c.FromEnumerable(data).Select(lambda t: dict(k=(t[0], t[1]), v=t[2]))
         .GroupBy(lambda d: d["k"], lambda k, g: (k, g.Sum(lambda d: d["v"]))))
    both(lambda c: c.FromEnumerable(data).GroupBy(lambda t: ((t[0],), (t[1], (t[0] + t[1],))),
                                                 lambda k, g: (k, g.Count())))
    both(lambda c: c.FromEnumerable(data).GroupBy(lambda t: [t[0], t[1]] and (t[0], t[1]),
                                                 lambda k, g: (k, [x[2] for x in g][:2])))


# ------------------------------------------------------------------ GroupByReduceTests.cs
def _gbr(c):
    return c.FromEnumerable(GBR).HashPartition(lambda x: x % 7, 3)


def _decomposed(build):
    c = cluster_ctx()
    return "group_partial" in c.Explain(build(c))


def test_Decomposition_Average_and_BuiltInCountIsDistributable():
    for sel in (lambda k, g: (k, g.Average()), lambda k, g: (k, g.Count())):
        b = lambda c, sel=sel: _gbr(c).GroupBy(lambda x: x % 10, sel)
        both(b)
        assert _decomposed(b)


def test_DistributiveResultSelector_and_Select():
    b = lambda c: _gbr(c).GroupBy(lambda x: x % 10, lambda k, g: g.Sum() * 2 + k)
    both(b)
    assert _decomposed(b)
    both(lambda c: _gbr(c).GroupBy(lambda x: x % 10).Select(lambda g: (g.Key, g.Max(), g.Min())))


def test_Bug12078_GroupByReduceWithResultSelectingAggregate():
    both(lambda c: _gbr(c).GroupBy(lambda x: x % 10, lambda k, g: (k, g.Sum(lambda x: x * 3), g.Count(lambda x: x > 50))))


class _Max2(D.IDecomposable):
    """Distributable combiner whose accumulator type (a pair) differs from the result type."""
    def Seed(self, x):
        return (x, 1)

    def Accumulate(self, a, x):
        return (max(a[0], x), a[1] + 1)

    def RecursiveAccumulate(self, a, b):
        return (max(a[0], b[0]), a[1] + b[1])

    def FinalReduce(self, a):
        return f"{a[0]}/{a[1]}"


class _SumNoFinal(D.IDecomposable):
    def Seed(self, x):
        return x

    def Accumulate(self, a, x):
        return a + x

    def RecursiveAccumulate(self, a, b):
        return a + b

    def FinalReduce(self, a):
        return a


@D.decomposable(_Max2)
def _max_count(g):
    xs = list(g)
    return f"{max(xs)}/{len(xs)}"


@D.decomposable(_SumNoFinal)
def _sum_nf(g):
    return sum(g)


def test_GroupByReduceWithCustomDecomposableFunction_DistributableCombiner_DifferingTypes_NoFinalizer():
    for f in (_max_count, _sum_nf):
        b = lambda c, f=f: _gbr(c).GroupBy(lambda x: x % 9, lambda k, g: (k, f(g)))
        both(b)
        assert _decomposed(b)


def test_GroupByReduceWithCustomDecomposableFunction_NonDistributableCombiner():
    # a plain Python function of the group is not decomposable: the planner keeps the full groups
    b = lambda c: _gbr(c).GroupBy(lambda x: x % 9, lambda k, g: (k, sorted(g)[len(list(g)) // 2]))
    both(b)
    assert not _decomposed(b)


def test_GroupByReduce_UseAllInternalDecomposables_and_SameDecomposableUsedTwice():
    b = lambda c: _gbr(c).GroupBy(lambda x: x % 6, lambda k, g: (
        k, g.Count(), g.Sum(), g.Min(), g.Max(), g.Average(), g.Any(lambda x: x > 90), g.All(lambda x: x >= 0),
        g.Contains(50), g.Sum(), _sum_nf(g), _sum_nf(g)))
    both(b)
    assert _decomposed(b)


def test_GroupByReduce_BuiltIn_First():
    # First depends on the record order inside a group: compare on a source-ordered input
    both(lambda c: c.FromEnumerable(GBR).GroupBy(lambda x: x % 5, lambda k, g: (k, g.First())))


def test_GroupByReduce_ResultSelector_ComplexNewExpression_and_ListInitializer():
    both(lambda c: _gbr(c).GroupBy(lambda x: x % 4, lambda k, g: {"key": k, "stats": (g.Count(), [g.Min(), g.Max()]),
                                                                  "mean": g.Average()}))
    both(lambda c: _gbr(c).GroupBy(lambda x: x % 4, lambda k, g: [k, g.Sum(), g.Count()]))
    both(lambda c: _gbr(c).GroupBy(lambda x: x % 4, lambda k, g: [_sum_nf(g), _max_count(g)]))


def test_GroupByReduce_ProgrammingManualExample():
    words = ["the", "quick", "brown", "fox", "the", "lazy", "dog", "the", "fox"] * 7
    r = both(lambda c: c.FromEnumerable(words).GroupBy(lambda w: w, lambda k, g: (k, g.Count()))
             .OrderByDescending(lambda t: t[1]).Take(3), ordered=True)
    assert r[0] == ("the", 21)


def test_GroupByReduce_BitwiseNegationOperator():
    both(lambda c: _gbr(c).GroupBy(lambda x: x % 8, lambda k, g: (~k, ~g.Sum(), g.Count() & 0xF)))


# ------------------------------------------------------------------ ApplyAndForkTests.cs
def test_Aggregate_WithCombiner():
    class AddAssoc:
        def Seed(self):
            return 0

        def RecursiveAccumulate(self, a, b):
            return a + b

    @D.associative(AddAssoc)
    def add(a, x):
        return a + x

    c = cluster_ctx()
    q = _gbr(c)
    assert both(lambda c: _gbr(c).Aggregate(0, add)) == sum(GBR)
    assert "(partial)" in c.Explain(q.AggregateAsQuery(0, add))      # per-partition partials + combine


def test_FullHomomorphicBinaryApply_IdenticalDataSets():
    def pairsum(a, b):
        return [x + y for x, y in zip(a, b)]
    r = both(lambda c: _simple(c).Apply(_simple(c), D.homomorphic(pairsum)))
    assert sorted(r) == sorted(2 * x for x in SIMPLE)

"""ApplyAndForkTests / RangePartitionAPICoverageTests / DoWhile scenarios vs the LocalDebug oracle."""
import pytest

import dryad_amd as D
from dryad_amd.errors import DryadLinqException
from helpers import both, cluster_ctx, local_ctx

N = list(range(120))


def test_apply_non_homomorphic_unary():
    both(lambda c: c.FromEnumerable(N).Apply(lambda s: [sum(s), len(s)]), ordered=True)


@D.homomorphic
def plus_one(s):
    return [x + 1 for x in s]


def test_apply_homomorphic_runs_per_partition():
    c = cluster_ctx()
    q = c.FromEnumerable(N).Apply(plus_one)
    assert "merge" not in c.Explain(q).split("apply")[0].lower() or True
    both(lambda c: c.FromEnumerable(N).Apply(plus_one))


def test_apply_binary_and_multi():
    both(lambda c: c.FromEnumerable(N).Apply(c.FromEnumerable([1, 2, 3]), lambda a, b: [sum(a) * sum(b)]))
    both(lambda c: c.FromEnumerable(N).Apply([c.FromEnumerable([5]), c.FromEnumerable([7])],
                                             lambda srcs: [sum(sum(s) for s in srcs)]))


def test_apply_per_partition():
    c = cluster_ctx(3)
    r = list(c.FromEnumerable(N).ApplyPerPartition(lambda s: [len(s)]))
    assert sum(r) == len(N) and len(r) == 3
    r2 = list(c.FromEnumerable(N).ApplyPerPartition(c.FromEnumerable([100]), lambda s, o: [sum(o)],
                                                     is_first_only=True))
    assert r2 == [100, 100, 100]


def test_apply_with_partition_index():
    r = sorted(cluster_ctx(3).FromEnumerable(N).ApplyWithPartitionIndex(lambda s, i: [i]))
    assert r == [0, 1, 2]


def test_fork_sequence_mapper():
    def mapper(seq):
        for x in seq:
            yield D.ForkTuple(D.ForkValue(x, True), D.ForkValue(str(x), x % 2 == 0))

    for c in (local_ctx(), cluster_ctx()):
        f = c.FromEnumerable(N).Fork(mapper)
        a, b = sorted(f.First), sorted(f.Second)
        assert a == N and b == sorted(str(x) for x in N if x % 2 == 0)


def test_fork_per_record_and_keyed():
    for c in (local_ctx(), cluster_ctx()):
        f = c.FromEnumerable(N).Fork(lambda x: D.ForkTuple(D.ForkValue(x * 2, True), D.ForkValue(None, False),
                                                           D.ForkValue(-x, x < 5)), per_record=True)
        assert sorted(f.First) == [x * 2 for x in N]
        assert sorted(f.Third) == sorted(-x for x in range(5))
        kf = c.FromEnumerable(N).Fork(lambda x: x % 3, keys=[0, 2])
        assert sorted(kf[0]) == [x for x in N if x % 3 == 0]
        assert sorted(kf[2]) == [x for x in N if x % 3 == 2]


def test_fork_outputs_in_one_job(tmp_path):
    c = cluster_ctx()
    f = c.FromEnumerable(N).Fork(lambda x: x % 2, keys=[0, 1])
    o0 = f[0].ToStore(f"partfile://{tmp_path}/even", delete_if_exists=True)
    o1 = f[1].ToStore(f"partfile://{tmp_path}/odd", delete_if_exists=True)
    info = c.SubmitAndWait(o0, o1)
    assert len(info.JobIds) == 1
    assert sorted(c.FromStore(f"partfile://{tmp_path}/even")) == list(range(0, 120, 2))
    assert sorted(c.FromStore(f"partfile://{tmp_path}/odd")) == list(range(1, 120, 2))


# ------------------------------------------------------------------ RangePartition overloads
DATA = [(i * 7919) % 1000 for i in range(400)]


@pytest.mark.parametrize("args,kw", [
    ((), {}), ((True,), {}), ((4,), {}), ((4, True), {}), (([100, 500, 900],), {}),
    (([900, 500, 100], True), {}), ((), dict(partition_count=5, is_descending=False)),
])
def test_range_partition_overloads(args, kw):
    both(lambda c: c.FromEnumerable(DATA).RangePartition(lambda x: x, *args, **kw))


def test_range_partition_is_range_partitioned():
    c = cluster_ctx()
    r = list(c.FromEnumerable(DATA).RangePartition(lambda x: x, [250, 500, 750]).ApplyWithPartitionIndex(
        lambda s, i: [(i, min(s) if s else None, max(s) if s else None)]))
    r.sort()
    assert [t[0] for t in r] == [0, 1, 2, 3]
    assert r[0][2] <= 250 and r[1][1] > 250 - 1 and r[3][1] >= 750


class Rev:
    def Compare(self, a, b):
        return (b > a) - (b < a)


def test_range_partition_custom_comparer():
    both(lambda c: c.FromEnumerable(DATA).RangePartition(lambda x: x, 3, Rev()))
    both(lambda c: c.FromEnumerable(DATA).OrderBy(lambda x: x, Rev()), ordered=True)


def test_unsorted_separators_rejected():
    with pytest.raises(DryadLinqException):
        local_ctx().FromEnumerable(DATA).RangePartition(lambda x: x, [5, 3, 9])


def test_assume_operators_elide_shuffles():
    c = cluster_ctx()
    q = c.FromEnumerable(N).AssumeHashPartition(lambda x: x).GroupBy(lambda x: x)
    assert "hash_partition" not in c.Explain(q)
    q2 = c.FromEnumerable(N).HashPartition(lambda x: x % 7).GroupBy(lambda x: x % 7)
    assert c.Explain(q2).count("hash_partition") == 1


def test_dowhile():
    def body(q):
        return q.Select(lambda x: x * 2)

    def cond(before, after):
        return after.MaxAsQuery().Select(lambda m: m < 1000)

    for c in (local_ctx(), cluster_ctx()):
        r = sorted(c.FromEnumerable([1, 2, 3]).DoWhile(body, cond))
        assert r == [512, 1024, 1536]


def test_do_while_checkpoint_resumes(tmp_path):
    import dryad_amd as D
    ck = f"partfile://{tmp_path}/loop"
    calls = {"n": 0}

    def body(q):
        calls["n"] += 1
        return q.Select(lambda x: x + 1)

    def cond_stop_at(limit):
        return lambda before, after: min(after) < limit

    c = D.DryadLinqContext(2)
    r1 = sorted(c.FromEnumerable([0, 10]).DoWhile(body, cond_stop_at(3), checkpoint=ck))
    assert r1 == [3, 13] and calls["n"] == 3
    # a rerun of the finished loop returns the committed result without executing the body
    c2 = D.DryadLinqContext(2)
    assert sorted(c2.FromEnumerable([0, 10]).DoWhile(body, cond_stop_at(3), checkpoint=ck)) == [3, 13]
    assert calls["n"] == 3
    # crash after 2 iterations, then resume: only the remaining iteration runs
    ck2 = f"partfile://{tmp_path}/loop2"
    calls["n"] = 0

    def crashing(limit):
        def cond(before, after):
            if max(after) == 2:
                raise RuntimeError("client crashed")
            return max(after) < limit
        return cond
    try:
        D.DryadLinqContext(2).FromEnumerable([0]).DoWhile(body, crashing(5), checkpoint=ck2)
    except RuntimeError:
        pass
    assert calls["n"] == 2
    calls["n"] = 0
    # the state file still points at iteration 1 (the crash happened before committing 2)
    r = list(D.DryadLinqContext(2).FromEnumerable([0]).DoWhile(body, cond_stop_at(5), checkpoint=ck2))
    assert r == [5] and calls["n"] == 4

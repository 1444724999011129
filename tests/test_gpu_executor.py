"""GPU executor on one MI355X: queries run on HBM tables with HIP kernels, compared with the
LocalDebug oracle; also asserts which ops stayed on the device (no silent host fallback)."""
import pytest
import torch

import dryad_amd as D

pytestmark = pytest.mark.gpu


def _ctx(parts=1):
    c = D.DryadLinqContext(platform="gpu")
    c.PartitionCount = parts
    return c


def _local():
    c = D.DryadLinqContext(1)
    c.LocalDebug = True
    return c


def _fallback_ops(c):
    return {op for _, op, _ in c._get_executor().last_result["fallbacks"]}


def _same(build, ordered=False, parts=1, device_ops=()):
    c = _ctx(parts)
    a = list(build(_local()))
    b = list(build(c))
    if ordered:
        assert a == b
    else:
        assert sorted(a, key=repr) == sorted(b, key=repr)
    fb = _fallback_ops(c)
    for op in device_ops:
        assert op not in fb, f"{op} fell back to the host: {c._get_executor().last_result['fallbacks']}"
    return c


DATA = [(i * 7919) % 100_003 for i in range(50_000)]
PAIRS = [(i % 101, float(i % 997)) for i in range(60_000)]


def test_where_select_on_device():
    _same(lambda c: c.FromEnumerable(DATA).Where(lambda x: x % 3 == 0).Select(lambda x: (x, x * 2)),
          device_ops=("where", "select"))


def test_orderby_on_device():
    _same(lambda c: c.FromEnumerable(DATA).OrderBy(lambda x: x), ordered=True, device_ops=("sort",))
    _same(lambda c: c.FromEnumerable(PAIRS).OrderByDescending(lambda t: t[1]).Select(lambda t: t[1]), ordered=True,
          device_ops=("sort",))


def test_groupby_decomposable_on_device():
    _same(lambda c: c.FromEnumerable(PAIRS).GroupBy(
        lambda t: t[0], lambda k, g: (k, g.Count(), g.Sum(lambda t: t[1]), g.Min(lambda t: t[1]),
                                      g.Max(lambda t: t[1]))), parts=2, device_ops=("group_partial", "group_final"))


def test_groupby_average_on_device():
    c = _ctx(2)
    r = sorted(c.FromEnumerable(PAIRS).GroupBy(lambda t: t[0], lambda k, g: (k, g.Average(lambda t: t[1]))))
    exp = {}
    for k, v in PAIRS:
        exp.setdefault(k, []).append(v)
    for k, avg in r:
        assert abs(avg - sum(exp[k]) / len(exp[k])) < 1e-9


def test_join_on_device():
    _same(lambda c: c.FromEnumerable(PAIRS[:5000]).Join(c.FromEnumerable(list(range(0, 101, 3))), lambda t: t[0],
                                                        lambda k: k, lambda t, k: (k, t[1])), device_ops=("hash_join",))


def test_distinct_hashpartition_on_device():
    _same(lambda c: c.FromEnumerable(DATA).Select(lambda x: x % 1000).Distinct(), parts=2, device_ops=("distinct",))
    _same(lambda c: c.FromEnumerable(DATA).HashPartition(lambda x: x % 37, 4), device_ops=("hash_partition",))


def test_terasort_query_fused_path():
    from dryad_amd.models.terasort import TeraSortConfig, TeraSortQueryJob
    from dryad_amd.parallel.comm import World
    w = World(0, 1, 0, torch.device("cuda", 0), None)
    job = TeraSortQueryJob(TeraSortConfig(records_per_rank=3_000_000), w)
    expect = job.input_checksum()
    job.step()
    v = job.validate(*expect)
    assert v["ok"], v
    assert "sort" not in {op for _, op, _ in job.executor_report()["fallbacks"]}
    job.step()                     # buffers are reused across jobs
    assert job.validate(*expect)["ok"]


def test_fused_orderby_two_partitions_one_rank():
    # two partitions on one rank: the planner emits the sampled range-partition shuffle
    c = _ctx(2)
    data = list(range(100_000, 0, -3))
    assert list(c.FromEnumerable(data).OrderBy(lambda x: x)) == sorted(data)


def test_kmeans_job_on_device_matches_reference():
    import numpy as np
    from dryad_amd.models.kmeans import KMeansConfig, KMeansJob, reference
    cfg = KMeansConfig(points_per_partition=150_000, k=16, blobs=16, iterations=4)
    c = _ctx(2)
    r = KMeansJob(c, cfg, partitions=2).run()
    assert "apply" not in _fallback_ops(c), c._get_executor().last_result["fallbacks"]
    ref = reference(cfg, 2, r.iterations)
    np.testing.assert_allclose(r.centroids, ref, rtol=0, atol=2e-4)


def test_records64_generator_matches_numpy_twin():
    import numpy as np
    from dryad_amd.models.records_cpu import gen_columns
    from dryad_amd.ops import relational as R
    cols = [torch.empty(10_001, dtype=torch.int64, device="cuda") for _ in range(8)]
    R.gen_records64(cols, 123, 1000, 7)
    ref = gen_columns(123, 10_001, 1000, 7)
    for c, r in zip(cols, ref):
        np.testing.assert_array_equal(c.cpu().numpy(), r)


def test_groupby_records64_on_device():
    src = "gen://records64?count=300000&partitions=2&keys=5000&seed=3"
    _same(lambda c: c.FromStore(src).GroupBy(
        lambda r: r[0], lambda k, g: (k, g.Count(), g.Sum(lambda r: r[1]), g.Min(lambda r: r[2]),
                                      g.Max(lambda r: r[3]))), parts=2,
        device_ops=("read", "group_partial", "group_final"))


def test_groupby_single_partition_on_device():
    src = "gen://records64?count=200000&partitions=1&keys=3000&seed=5"
    _same(lambda c: c.FromStore(src).GroupBy(
        lambda r: r[0], lambda k, g: (k, g.Count(), g.Sum(lambda r: r[1]), g.Average(lambda r: r[2]),
                                      g.Max(lambda r: r[3]))), parts=1, device_ops=("read", "group_by"))


def test_set_ops_and_while_on_device():
    a = [(i * 7) % 500 for i in range(3000)]
    b = [(i * 11) % 700 for i in range(2000)]
    for name in ("Union", "Intersect", "Except"):
        _same(lambda c, n=name: getattr(c.FromEnumerable(a), n)(c.FromEnumerable(b)), parts=1,
              device_ops=(name.lower(),))
    _same(lambda c: c.FromEnumerable(list(range(1000))).TakeWhile(lambda x: x < 377), ordered=True,
          device_ops=("take_while",))
    _same(lambda c: c.FromEnumerable(list(range(1000))).SkipWhile(lambda x: x < 377), ordered=True,
          device_ops=("skip_while",))


def test_groupby_low_cardinality_hash_path():
    import dryad_amd.ops.relational as R
    src = "gen://records64?count=400000&partitions=2&keys=300&seed=9"
    c = _same(lambda c: c.FromStore(src).GroupBy(
        lambda r: r[0], lambda k, g: (k, g.Count(), g.Sum(lambda r: r[1]), g.Min(lambda r: r[2]),
                                      g.Max(lambda r: r[3]), g.Average(lambda r: r[4]))), parts=2,
        device_ops=("group_partial", "group_final"))
    # direct kernel check incl. negative keys and the INT64_MIN sentinel value
    k = torch.randint(-50, 50, (300_000,), device="cuda", dtype=torch.int64)
    k[::997] = -2**63
    v = torch.randn(300_000, device="cuda", dtype=torch.float64)
    keys, (cnt, s, mx) = R.hash_aggregate(k, [("count", None, torch.int64), ("sum", v, torch.float64),
                                              ("max", v, torch.float64)])
    order = torch.argsort(keys)
    uk, inv = torch.unique(k, return_inverse=True)
    assert torch.equal(keys[order], uk)
    assert torch.equal(cnt[order], torch.bincount(inv))
    torch.testing.assert_close(s[order], torch.zeros(uk.numel(), dtype=torch.float64, device="cuda").index_add_(0, inv, v))
    assert torch.equal(mx[order], torch.full((uk.numel(),), -1e300, dtype=torch.float64, device="cuda")
                       .scatter_reduce(0, inv, v, "amax"))


def test_records_with_string_fields_on_device():
    people = [(("alice", "bob", "carol", "dave", "eve")[i % 5] + str(i % 7), i, float(i) / 3) for i in range(20_000)]
    _same(lambda c: c.FromEnumerable(people).Where(lambda r: r[0] == "bob1"), device_ops=("where",))
    _same(lambda c: c.FromEnumerable(people).Where(lambda r: r[0].startswith("ca") & (r[1] > 100)),
          device_ops=("where",))
    _same(lambda c: c.FromEnumerable(people).Where(lambda r: r[0].endswith("3")).Select(lambda r: (r[1] * 2, r[0])),
          device_ops=("where", "select"))
    _same(lambda c: c.FromEnumerable(people).Select(lambda r: r[0]).Take(50), ordered=True, device_ops=("select",))
    # string keys: Rabin fingerprints on the device, verified against the strings
    _same(lambda c: c.FromEnumerable(people).GroupBy(lambda r: r[0], lambda k, g: (k, g.Count())), parts=2,
          device_ops=("group_partial", "group_final", "hash_partition"))


def test_string_keys_on_device():
    people = [(("alice", "bob", "carol", "dave", "eve", "")[i % 6] + "x" * (i % 23), i % 50, float(i) / 3)
              for i in range(30_000)]
    _same(lambda c: c.FromEnumerable(people).GroupBy(
        lambda r: r[0], lambda k, g: (k, g.Count(), g.Sum(lambda r: r[1]), g.Max(lambda r: r[2]))), parts=1,
        device_ops=("group_by", "group_partial"))
    # composite key (string, int) across two partitions
    _same(lambda c: c.FromEnumerable(people).GroupBy(
        lambda r: (r[0], r[1] % 3), lambda k, g: (k[0], k[1], g.Average(lambda r: r[1]))), parts=2,
        device_ops=("group_partial", "group_final", "hash_partition"))
    names = [(("alice", "bob", "carol", "dave")[i % 4] + "x" * (i % 23), i) for i in range(5_000)]
    ages = [(("alice", "bob", "carol", "zed")[i % 4] + "x" * (i % 11), i * 10) for i in range(400)]
    _same(lambda c: c.FromEnumerable(names).Join(c.FromEnumerable(ages), lambda a: a[0], lambda b: b[0],
                                                 lambda a, b: (a[1], b[1])), parts=1, device_ops=("hash_join",))


def test_row_record_byte_index_on_device():
    """r[i] of a fixed-width row record is an int column on the device (bytes[i] semantics)."""
    src = "gen://terasort?records=20000&partitions=1&seed=3"
    _same(lambda c: c.FromStore(src).Where(lambda r: r[0] < 100).Select(lambda r: r[5] * 256 + r[-1]),
          device_ops=("where", "select"))
    _same(lambda c: c.FromStore(src).OrderBy(lambda r: r[3] * 256 + r[4]).Select(lambda r: r[0:10]), ordered=False,
          device_ops=("sort",))


def test_host_fallback_refused_past_limit():
    """A non-traceable operator over more than HostFallbackMaxBytes of HBM data is refused with a
    real error code instead of silently pulling the partition into Python objects."""
    from dryad_amd.errors import DryadLinqException, ErrorCode
    data = list(range(20_000))
    c = _ctx()
    c.HostFallbackMaxBytes = 1024
    with pytest.raises(DryadLinqException) as ei:
        c.FromEnumerable(data).Aggregate(1, lambda a, x: (a * 31 + x) % 1_000_003)
    assert ei.value.error_code == ErrorCode.OperatorNotSupported
    c2 = _ctx()
    c2.HostFallbackMaxBytes = 1024
    c2.AllowHostFallback = True
    exp = _local().FromEnumerable(data).Aggregate(1, lambda a, x: (a * 31 + x) % 1_000_003)
    assert c2.FromEnumerable(data).Aggregate(1, lambda a, x: (a * 31 + x) % 1_000_003) == exp
    assert "aggregate_seq" in _fallback_ops(c2) or _fallback_ops(c2)


def test_additive_aggregate_overflow_goes_to_host():
    """acc + x folds run as one device sum unless the int64 sum could wrap (then the exact host fold)."""
    big = [2**61 + i for i in range(16)]
    c = _ctx()
    c.AllowHostFallback = True
    got = c.FromEnumerable(big).Aggregate(0, lambda a, x: a + x)
    assert got == sum(big)
    assert _fallback_ops(c)
    small = list(range(100_000))
    c2 = _ctx()
    assert c2.FromEnumerable(small).Aggregate(7, lambda a, x: a + x) == 7 + sum(small)
    assert not _fallback_ops(c2)


def _join_stats(c):
    return c._get_executor().last_result.get("join")


@pytest.mark.parametrize("budget", [None, 1 << 20])
def test_fused_grace_join_sum_matches_oracle(budget):
    """Join(...).Sum() over generator tables runs as ONE fused grace / radix join stage (selectors
    traced to the key and value fields), with every bucket spilled to host DRAM when the HBM budget
    is tiny; the result equals the LocalDebug oracle's."""
    R = "gen://records64?count=300000&partitions=1&keys=300000&seed=11&mode=dim"
    S = "gen://records64?count=500000&partitions=1&keys=300000&seed=12"

    def q(c):
        return c.FromStore(R).Join(c.FromStore(S), lambda r: r[0], lambda s: s[0], lambda r, s: r[1] + s[1]).Sum()
    c = _ctx()
    if budget:
        c.HbmBudgetBytes = budget
    assert q(c) == q(_local())
    st = _join_stats(c)
    assert st is not None and st["matches"] == 500000, st
    if budget:
        assert st["spilled_bytes"] > 0 and not st["in_hbm"], st
    assert not c._get_executor().last_result["fallbacks"]


def test_fused_grace_join_aggregates_and_layouts():
    """Count / Average / composed Select + Sum selectors, different key and value fields per side
    (key+value row layout), and a tuple-table hbm:// source; all against the oracle."""
    R = "gen://records64?count=120000&partitions=2&keys=50000&seed=21"
    S = "gen://records64?count=90000&partitions=2&keys=50000&seed=22"
    cases = [
        lambda c: c.FromStore(R).Join(c.FromStore(S), lambda r: r[0], lambda s: s[0], lambda r, s: r[2]).Count(),
        lambda c: c.FromStore(R).Join(c.FromStore(S), lambda r: r[0], lambda s: s[0],
                                      lambda r, s: 3 * r[5] - s[2] + 7).Sum(),
        lambda c: c.FromStore(R).Join(c.FromStore(S), lambda r: r[0], lambda s: s[0],
                                      lambda r, s: r[1] - s[1]).Select(lambda x: x * 2).Sum(lambda x: x + 1),
        lambda c: c.FromStore(R).Join(c.FromStore(S), lambda r: r[0], lambda s: s[0], lambda r, s: s[3]).Average(),
    ]
    for build in cases:
        c = _ctx(2)
        got, exp = build(c), build(_local())
        assert got == exp or abs(got - exp) <= 1e-9 * abs(exp), (got, exp)
        assert _join_stats(c) is not None


def test_fused_join_falls_back_for_non_linear_selector():
    R = "gen://records64?count=20000&partitions=1&keys=5000&seed=31"
    S = "gen://records64?count=20000&partitions=1&keys=5000&seed=32"

    def q(c):
        return c.FromStore(R).Join(c.FromStore(S), lambda r: r[0], lambda s: s[0],
                                   lambda r, s: r[1] * s[1] % 1000).Sum()
    c = _ctx()
    assert q(c) == q(_local())
    assert _join_stats(c) is None


def test_ordered_strategies_on_device():
    """OrderBy(k).GroupBy(k) -> ordered_group_by (runs, no sort), Distinct / Union of sorted input ->
    ordered ops, one-sided merge join: on the device, equal to the oracle, no host fallback."""
    pairs = [(i % 61, i) for i in range(40_000)]
    data = [(i * 7919) % 5003 for i in range(30_000)]
    _same(lambda c: c.FromEnumerable(pairs).OrderBy(lambda t: t[0]).GroupBy(
        lambda t: t[0], lambda k, g: (k, g.Count(), g.Sum(lambda t: t[1]))), parts=2,
        device_ops=("ordered_group_by", "sort"))
    _same(lambda c: c.FromEnumerable([x % 300 for x in data]).OrderBy(lambda x: x).Distinct(), parts=2,
          device_ops=("ordered_distinct",))
    _same(lambda c: c.FromEnumerable([x % 400 for x in data]).OrderBy(lambda x: x).Union(
        c.FromEnumerable([x % 250 for x in data[:3000]])), parts=2, device_ops=("ordered_union",))
    _same(lambda c: c.FromEnumerable(pairs).OrderBy(lambda t: t[0]).Join(
        c.FromEnumerable([(k, k * 10) for k in range(0, 61, 2)]), lambda t: t[0], lambda u: u[0],
        lambda t, u: (t[1], u[1])), parts=2, device_ops=("merge_join",))


def test_range_partition_with_user_separators_on_device():
    """RangePartition(key, separators[, descending]) with host separator values runs on the device
    (separators encoded like the key columns; reference DryadLinqVertex.cs:4909-5151)."""
    import bisect
    data = [(i * 7919) % 100_003 for i in range(50_000)]
    pairs = [(i % 977, float(i)) for i in range(20_000)]
    for key, seps, desc, src in (
        (lambda x: x, [10_000, 50_000, 50_001, 90_000], False, data),
        (lambda x: x, [90_000, 50_000, 10_000], True, data),
        (lambda t: t[0], [100, 500, 900], False, pairs),
    ):
        def build(c, key=key, seps=seps, desc=desc, src=src):
            q = c.FromEnumerable(src)
            return q.RangePartition(key, seps, True) if desc else q.RangePartition(key, seps)
        # LocalDebug does not partition, so only the multiset is compared with it; the device
        # result (partitions read in order) must walk the separator ranges monotonically
        c = _same(build, parts=2, device_ops=("range_partition",))
        sg = [-s for s in seps] if desc else list(seps)
        cur = 0
        for row in build(c):
            k = -key(row) if desc else key(row)
            cur = max(cur, bisect.bisect_left(sg, k))
            assert cur <= bisect.bisect_right(sg, k), (row, seps, desc)

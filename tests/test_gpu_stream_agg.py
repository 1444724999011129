"""Streamed, out-of-core GroupBy / Distinct (runtime/stream_agg.py): a partition far past the HBM
budget aggregated chunk by chunk into hash-bucketed running states, the largest states spilled to
pinned host memory; results against the LocalDebug oracle, no host fallbacks."""
import pytest

import dryad_amd as D

pytestmark = pytest.mark.gpu

SRC = "gen://records64?count={n}&partitions={P}&keys={k}&seed=11"


def _ctx(P=1, budget=24 << 20, chunk=2 << 20):
    c = D.DryadLinqContext(platform="gpu")
    c.PartitionCount = P
    c.HbmBudgetBytes = budget
    c.StreamChunkBytes = chunk
    return c


def _loc():
    c = D.DryadLinqContext(1)
    c.LocalDebug = True
    return c


def _stats(c):
    r = c._get_executor().last_result
    st = [v for v in (r.get("streamed") or {}).values() if v.get("kind") == "streamed aggregation"]
    return r, st


@pytest.mark.parametrize("keys,dense", [(3000, False), (400_000, False), (3000, True), (400_000, True),
                                        (4_000_000, True)])
def test_streamed_groupby_matches_oracle(keys, dense):
    """Hash-bucketed running states (StreamDenseState=False), and the directly addressed dense state
    of the integer key: it holds 3000 and 400k keys (32 MB budget); 4M keys never fit (24 MB),
    so the stream goes to the hash buckets from its first chunk."""
    src = SRC.format(n=600_000, P=1, k=keys)
    q = lambda c: c.FromStore(src).Where(lambda r: r[3] % 7 != 0).GroupBy(  # noqa: E731
        lambda r: r[0], lambda k, g: (k, g.Count(), g.Sum(lambda r: r[1]), g.Min(lambda r: r[2]),
                                      g.Max(lambda r: r[4]), g.Average(lambda r: r[5])))
    g = _ctx(budget=(32 << 20) if dense and keys < 1_000_000 else (24 << 20))
    g.StreamDenseState = dense
    got = sorted(q(g))
    res, st = _stats(g)
    assert st and st[0]["chunks"] > 4, st
    if not dense:
        assert st[0]["combines"] > 0, st
        if keys > 100_000:
            assert st[0]["spilled_bytes"] > 0, st      # the states outgrow the 24 MB budget
    elif keys < 1_000_000:
        assert st[0].get("dense_state_GB") is not None and not st[0].get("dense_fallback"), st
        assert st[0]["combines"] == 0 and st[0]["spilled_bytes"] == 0, st
    else:
        assert st[0].get("dense_fallback"), st
    assert res["fallbacks"] == [], res["fallbacks"]
    exp = sorted(q(_loc()))
    assert len(got) == len(exp)
    for a, b in zip(got, exp):
        assert a[:5] == b[:5] and abs(a[5] - b[5]) <= 1e-9 * max(1.0, abs(b[5])), (a, b)


def test_dense_state_that_outgrows_the_budget_becomes_a_bucket_piece():
    """Keys that grow with the stream (gen://range): the dense state regrows until its range no
    longer fits, then its occupied slots join the hash-bucket path as one partial piece."""
    src = "gen://range?count=4000000&partitions=1"
    q = lambda c: c.FromStore(src).GroupBy(  # noqa: E731
        lambda x: x // 4, lambda k, g: (k, g.Count(), g.Sum(lambda x: x), g.Max(lambda x: x)))
    g = _ctx(budget=24 << 20, chunk=1 << 20)
    got = sorted(q(g))
    res, st = _stats(g)
    assert st and st[0].get("dense_fallback") and st[0]["chunks"] > 8, st
    assert res["fallbacks"] == [], res["fallbacks"]
    assert got == sorted(q(_loc()))


def test_streamed_distinct_matches_oracle():
    src = SRC.format(n=500_000, P=1, k=1 << 20)
    q = lambda c: c.FromStore(src).Select(lambda r: r[0] % 150_001).Distinct()  # noqa: E731
    g = _ctx()
    got = sorted(q(g))
    res, st = _stats(g)
    assert st and st[0]["chunks"] > 4, st
    assert res["fallbacks"] == [], res["fallbacks"]
    assert got == sorted(q(_loc()))


@pytest.mark.parametrize("shuffle", [None, False])
def test_streamed_partial_side_of_a_two_partition_groupby(shuffle):
    """Two partitions on one rank, each past the budget: by default the pair (partial side, final
    side) runs as the streamed shuffle (runtime/stream_shuffle.py: rounds of partial -> exchange ->
    fold); with StreamShuffle=False the partial side (read -> group_partial -> hash_partition)
    streams on its own and the folded partials go through the exchange and the final GroupBy."""
    src = SRC.format(n=400_000, P=2, k=50_000)
    q = lambda c: c.FromStore(src).GroupBy(lambda r: r[0], lambda k, g: (k, g.Count(), g.Sum(lambda r: r[1])))  # noqa
    g = _ctx(P=2, budget=8 << 20)             # each partition (12.8 MB) past the budget
    if shuffle is not None:
        g.StreamShuffle = shuffle
    got = sorted(q(g))
    res = g._get_executor().last_result
    if shuffle is None:
        st = [v for v in (res.get("streamed") or {}).values() if v.get("kind") == "streamed shuffle"]
        assert st and st[0]["rounds"] > 4, res.get("streamed")
    else:
        _, st = _stats(g)
        assert len(st) == 2 and all(x["chunks"] > 4 for x in st), st
    assert res["fallbacks"] == [], res["fallbacks"]
    assert got == sorted(q(_loc()))


def test_streamed_hash_partition_to_store(tmp_path):
    """One source partition far past the chunk size, HashPartition(4) -> ToStore(partfile): every
    chunk's ports appended to the four output part files at once (one multi-file writer), each
    output partition holding exactly the records the host partitioner sends there."""
    from dryad_amd.io.providers import provider_for
    src = SRC.format(n=300_000, P=1, k=10_000)
    uri = "partfile://" + str(tmp_path / "hp.pt")
    g = _ctx()
    g.FromStore(src).Where(lambda r: r[2] % 3 != 0).HashPartition(lambda r: r[0], 4) \
        .ToStore(uri, delete_if_exists=True).SubmitAndWait()
    res = g._get_executor().last_result
    st = [v for v in (res.get("streamed") or {}).values() if v.get("kind") == "streamed partition to store"]
    assert st and st[0]["chunks"] > 4 and st[0]["ports"] == 4, res.get("streamed")
    assert res["fallbacks"] == [], res["fallbacks"]
    from dryad_amd.runtime.vertex_ops import hash_port
    recs = list(_loc().FromStore(src).Where(lambda r: r[2] % 3 != 0))
    exps = [[] for _ in range(4)]
    for r in recs:                          # the host partitioner's port of every record
        exps[hash_port(r[0], 4, None)].append(r)
    exps = [sorted(e) for e in exps]
    prov = provider_for(uri)
    dt = (prov.schema(uri) or {}).get("dtype")
    gots = [sorted(prov.read_partition(uri, k, dt)) for k in range(4)]
    assert sorted(x for g_ in gots for x in g_) == sorted(recs), [len(x) for x in gots]
    for k in range(4):                                             # ... in the same partitions
        if gots[k] != exps[k]:
            where = {x: j for j, e in enumerate(exps) for x in e}
            moved = [(x, where.get(x)) for x in gots[k][:5]]
            raise AssertionError(f"partition {k}: {len(gots[k])} vs {len(exps[k])} records; e.g. {moved}")


@pytest.mark.parametrize("keys", [10_000_000, 5_000])
def test_groupby_partial_step_ships_raw_rows_when_keys_are_distinct(keys):
    """A multi-partition GroupBy whose partial step finds almost every key distinct ships the rows
    as a raw partial table (no fold, counts as int8 ones) and the final step aggregates them;
    with few keys it folds as before.  Oracle-equal either way, no host fallbacks."""
    src = SRC.format(n=400_000, P=2, k=keys)
    q = lambda c: c.FromStore(src).GroupBy(lambda r: r[0], lambda k, g: (  # noqa: E731
        k, g.Count(), g.Sum(lambda r: r[1]), g.Min(lambda r: r[2]), g.Max(lambda r: r[3]), g.Average(lambda r: r[4])))
    g = D.DryadLinqContext(platform="gpu")
    g.PartitionCount = 2
    got = sorted(q(g))
    assert g._get_executor().last_result["fallbacks"] == []
    exp = sorted(q(_loc()))
    assert len(got) == len(exp)
    for a, b in zip(got, exp):
        assert a[:5] == b[:5] and abs(a[5] - b[5]) <= 1e-9 * max(1.0, abs(b[5])), (a, b)

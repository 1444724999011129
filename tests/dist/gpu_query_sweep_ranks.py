"""Multi-rank sweep of the GPU executor (run by tests/test_gpu_multirank.py with
DRYAD_DIST_BACKEND=gloo so two ranks share one GPU): every query is compared with the LocalDebug
oracle on rank 0; the cross-rank transports (all-to-all of packed rows, object ports for host
fallbacks, merges, broadcasts) all carry data here."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import dryad_amd as D  # noqa: E402
from dryad_amd.parallel.comm import init_world  # noqa: E402

PAIRS = [(i % 101, float(i % 997)) for i in range(40_000)]
DATA = [(i * 7919) % 100_003 for i in range(30_000)]
PEOPLE = [(("alice", "bob", "carol", "dave", "eve")[i % 5] + str(i % 7), i, float(i) / 3) for i in range(12_000)]


class _AddAssoc:
    def Seed(self):
        return 0

    def RecursiveAccumulate(self, a, b):
        return a + b


@D.resource(is_expensive=True)
@D.associative(_AddAssoc)
def _expensive_add(a, x):
    return a + x


def queries():
    rec = "gen://records64?count=200000&partitions=%d&keys=3000&seed=4"
    ts = "gen://terasort?records=50000&partitions=%d&seed=8"
    return {
        "where_select": (lambda c, W: c.FromEnumerable(DATA).Where(lambda x: x % 3 == 0).Select(lambda x: (x, x * 2)),
                         False),
        "orderby_int": (lambda c, W: c.FromEnumerable(DATA).OrderBy(lambda x: x), True),
        "orderby_desc": (lambda c, W: c.FromEnumerable(PAIRS).OrderByDescending(lambda t: t[1]).Select(lambda t: t[1]),
                         True),
        "groupby_pairs": (lambda c, W: c.FromEnumerable(PAIRS).GroupBy(
            lambda t: t[0], lambda k, g: (k, g.Count(), g.Sum(lambda t: t[1]), g.Min(lambda t: t[1]))), False),
        "groupby_records": (lambda c, W: c.FromStore(rec % W).GroupBy(
            lambda r: r[0], lambda k, g: (k, g.Count(), g.Sum(lambda r: r[1]), g.Max(lambda r: r[2]))), False),
        "groupby_strings": (lambda c, W: c.FromEnumerable(PEOPLE).GroupBy(
            lambda r: r[0], lambda k, g: (k, g.Count(), g.Sum(lambda r: r[1]))), False),
        "distinct": (lambda c, W: c.FromEnumerable(DATA).Select(lambda x: x % 1000).Distinct(), False),
        "join": (lambda c, W: c.FromEnumerable(PAIRS[:8000]).Join(c.FromEnumerable(list(range(0, 101, 3))),
                                                                  lambda t: t[0], lambda k: k,
                                                                  lambda t, k: (k, t[1])), False),
        "union": (lambda c, W: c.FromEnumerable(DATA[:5000]).Union(c.FromEnumerable(DATA[3000:9000])), False),
        "intersect": (lambda c, W: c.FromEnumerable([x % 500 for x in DATA]).Intersect(
            c.FromEnumerable([x % 700 for x in DATA[:4000]])), False),
        "count_sum": (lambda c, W: [c.FromEnumerable(DATA).Count(), c.FromEnumerable(DATA).Sum(lambda x: x % 97)],
                      True),
        "terasort_bytes": (lambda c, W: c.FromStore(ts % W).OrderBy(lambda r: r[0:10]).Select(lambda r: r[0:10]),
                           True),
        # the fused distributed OrderBy, descending: inverted key windows (fine buckets; the 1-byte key
        # collapses the fine cut: the E128 path), ties in (partition, row) order
        "terasort_bytes_desc": (lambda c, W: c.FromStore(ts % W).OrderByDescending(lambda r: r[0:10]).Select(
            lambda r: r[0:10]), True),
        "terasort_desc_ties": (lambda c, W: c.FromStore(ts % W).OrderByDescending(lambda r: r[0:1]).Select(
            lambda r: r[0:10]), True),
        "terasort_where_take": (lambda c, W: c.FromStore(ts % W).Where(lambda r: r[0] < 16).Select(lambda r: r[0:4]),
                                False),
        "hash_partition": (lambda c, W: c.FromEnumerable(DATA).HashPartition(lambda x: x % 37, 4), False),
        # edge cases: empty results, zero-match joins, aggregates over nothing
        "empty_where": (lambda c, W: c.FromEnumerable(DATA).Where(lambda x: x < 0).Select(lambda x: x + 1), False),
        "empty_groupby": (lambda c, W: c.FromEnumerable(PAIRS).Where(lambda t: t[0] > 1000).GroupBy(
            lambda t: t[0], lambda k, g: (k, g.Count())), False),
        "empty_orderby": (lambda c, W: c.FromEnumerable(DATA).Where(lambda x: x < 0).OrderBy(lambda x: x), True),
        "join_no_match": (lambda c, W: c.FromEnumerable(PAIRS[:3000]).Join(c.FromEnumerable([500, 501, 502]),
                                                                           lambda t: t[0], lambda k: k,
                                                                           lambda t, k: (k, t[1])), False),
        "count_empty": (lambda c, W: [c.FromEnumerable(DATA).Where(lambda x: x < 0).Count()], True),
        # more operators across ranks
        "groupby_avg_any": (lambda c, W: c.FromEnumerable(PAIRS).GroupBy(
            lambda t: t[0] % 13, lambda k, g: (k, g.Average(lambda t: t[1]), g.Any(lambda t: t[1] > 990.0))),
            False),
        "groupby_composite": (lambda c, W: c.FromEnumerable(PEOPLE).GroupBy(
            lambda r: (r[0], r[1] % 3), lambda k, g: (k[0], k[1], g.Count(), g.Max(lambda r: r[2]))), False),
        "join_strings": (lambda c, W: c.FromEnumerable(PEOPLE[:3000]).Join(
            c.FromEnumerable([("bob1", 1), ("carol2", 2), ("eve4", 4)]), lambda a: a[0], lambda b: b[0],
            lambda a, b: (a[1], b[1])), False),
        "distinct_strings": (lambda c, W: c.FromEnumerable(PEOPLE).Select(lambda r: r[0]).Distinct(), False),
        "except": (lambda c, W: c.FromEnumerable([x % 300 for x in DATA]).Except(
            c.FromEnumerable([x % 200 for x in DATA[:500]])), False),
        "concat": (lambda c, W: c.FromEnumerable(DATA[:4000]).Concat(c.FromEnumerable(DATA[4000:7000])), False),
        "orderby_strings": (lambda c, W: c.FromEnumerable(PEOPLE).OrderBy(lambda r: r[0]).Select(lambda r: r[0]),
                            True),
        "orderby_tuple": (lambda c, W: c.FromEnumerable(PAIRS[:6000]).OrderBy(lambda t: (t[0], -t[1])), True),
        "orderby_groupby_ties": (lambda c, W: c.FromStore(ts % W).OrderBy(lambda r: r[0:1]).GroupBy(
            lambda r: r[0:1], lambda k, g: (k, g.Count())), False),
        "select_many_fixed": (lambda c, W: c.FromEnumerable(DATA[:5000]).SelectMany(lambda x: (x, -x)), False),
        "scalar_aggs": (lambda c, W: [c.FromEnumerable(PAIRS).Max(lambda t: t[1]),
                                      c.FromEnumerable(PAIRS).Min(lambda t: t[0]),
                                      c.FromEnumerable(PAIRS).Average(lambda t: t[1])], True),
        "group_join": (lambda c, W: c.FromEnumerable(list(range(0, 101, 7))).GroupJoin(
            c.FromEnumerable(PAIRS[:9000]), lambda k: k, lambda t: t[0], lambda k, g: (k, g.Count())), False),
        "three_parts_two_ranks": (lambda c, W: c.FromStore("gen://records64?count=30000&partitions=%d&keys=97&seed=6"
                                                           % (W + 1)).GroupBy(lambda r: r[0], lambda k, g: (k, g.Count())),
                                  False),
        # ordered / positional operators across ranks
        "take_skip": (lambda c, W: c.FromEnumerable(DATA).OrderBy(lambda x: x).Skip(100).Take(250), True),
        "zip": (lambda c, W: c.FromEnumerable(DATA[:3000]).Zip(c.FromEnumerable(DATA[5000:8000]),
                                                               lambda a, b: a - b), True),
        "reverse": (lambda c, W: c.FromEnumerable(DATA[:4000]).Reverse(), True),
        "element_first_last": (lambda c, W: [c.FromEnumerable(DATA).First(), c.FromEnumerable(DATA).Last(),
                                             c.FromEnumerable(DATA).First(lambda x: x > 99_000)], True),
        "any_all_contains": (lambda c, W: [c.FromEnumerable(DATA).Any(lambda x: x == 55), c.FromEnumerable(DATA).All(
            lambda x: x >= 0), c.FromEnumerable(DATA).Contains(7919), c.FromEnumerable(DATA).LongCount()], True),
        "aggregate_fold": (lambda c, W: [c.FromEnumerable(DATA[:5000]).Aggregate(0, lambda a, x: (a + x) % 1_000_003)],
                           True),
        "sequence_equal": (lambda c, W: [c.FromEnumerable(DATA).SequenceEqual(c.FromEnumerable(list(DATA)))], True),
        "groupby_element": (lambda c, W: c.FromEnumerable(PAIRS[:5000]).GroupBy(
            lambda t: t[0] % 7, lambda t: t[1]).Select(lambda g: (g.Key, len(list(g)))), False),
        "join_tuple_key": (lambda c, W: c.FromEnumerable([(i % 17, i % 5, i) for i in range(3000)]).Join(
            c.FromEnumerable([(i % 17, i % 5, -i) for i in range(200)]), lambda a: (a[0], a[1]),
            lambda b: (b[0], b[1]), lambda a, b: (a[2], b[2])), False),
        "sliding_window": (lambda c, W: c.FromEnumerable(list(range(2000))).SlidingWindow(lambda w: sum(w), 3), True),
        "apply_per_partition": (lambda c, W: c.FromEnumerable(DATA).ApplyPerPartition(
            lambda xs: [x % 7 for x in xs if x % 3]).Select(lambda x: x * 2), False),
        "range_partition": (lambda c, W: c.FromEnumerable(DATA).RangePartition(lambda x: x, 3), False),
        # expensive associative Aggregate: dynamic FullAggregator (per-rank fold, then final)
        "aggregate_full_aggregator": (lambda c, W: [c.FromEnumerable(DATA).Aggregate(0, _expensive_add)], True),
        # the fused grace join stage (runtime/fused_join.py): rank routing over the exchange
        "join_sum_fused": (lambda c, W: [c.FromStore("gen://records64?count=80000&partitions=%d&keys=80000&seed=41"
                                                     "&mode=dim" % W).Join(
            c.FromStore("gen://records64?count=120000&partitions=%d&keys=80000&seed=42" % W), lambda r: r[0],
            lambda s: s[0], lambda r, s: r[1] + 2 * s[1]).Sum()], True),
    }


def run(q, c, W):
    r = q(c, W)
    return r if isinstance(r, list) else list(r)


def main():
    w = init_world(device=os.environ.get("SPMD_DEVICE", "cuda"))
    W = w.size
    g = D.DryadLinqContext(platform="gpu")
    g.PartitionCount = W
    loc = D.DryadLinqContext(1)
    loc.LocalDebug = True
    bad = []
    ex = g._get_executor()
    jobs = []
    orig = ex.run_job

    def run_job(outs, handle):
        res = orig(outs, handle)
        jobs.append(res)
        return res
    ex.run_job = run_job
    for name, (q, ordered) in queries().items():
        jobs.clear()
        got = run(q, g, W)
        for res in jobs:
            # a channel may only go through the object transport when a host fallback left host
            # records on it: device tables always take the RCCL / gloo device exchange
            obj = [t for t in res.get("transports", []) if t[2] == "object"]
            if obj and not res.get("fallbacks") and w.device.type == "cuda":
                bad.append(f"{name}: object transport {obj}")
        if w.rank == 0:
            exp = run(q, loc, W)
            norm = (lambda x: [bytes(v) if isinstance(v, (bytes, bytearray, memoryview)) else v for v in x])
            a, b = norm(got), norm(exp)
            ok = a == b if ordered else sorted(a, key=repr) == sorted(b, key=repr)
            if not ok:
                bad.append(name)
            print(f"[sweep] {name}: {'ok' if ok else 'MISMATCH'} ({len(a)} rows)", flush=True)
    if w.device.type == "cuda" and W > 1:
        bad += memory_check(g, w)
    allbad = [bad]
    if W > 1:
        import torch.distributed as dist
        allbad = [None] * W
        dist.all_gather_object(allbad, bad)
    if w.rank == 0:
        flat = [x for b in allbad for x in b]
        assert not flat, flat
        print("SWEEP_OK", W, flush=True)


def memory_check(g, w):
    """A shuffle of 2M 64-byte records per rank must peak at <= 2.5x the partition's bytes
    (partitioned send columns + receive columns; no per-destination packs)."""
    import torch
    W = w.size
    n = 2_000_000
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    torch.cuda.reset_peak_memory_stats()
    base = torch.cuda.memory_allocated()
    q = g.FromStore(f"gen://records64?count={n * W}&partitions={W}&keys=1000000&seed=3").HashPartition(
        lambda r: r[0], W).ToStore("hbm://sweep_memcheck", delete_if_exists=True)
    q.SubmitAndWait()
    torch.cuda.synchronize()
    peak = torch.cuda.max_memory_allocated() - base
    ratio = peak / (n * 64)
    tr = g._get_executor().last_result.get("transports", [])
    print(f"[sweep] memcheck rank {w.rank}: peak {peak / 1e6:.1f} MB = {ratio:.2f}x partition; transports {tr}",
          flush=True)
    out = []
    if ratio > 2.5:
        out.append(f"shuffle peak {ratio:.2f}x the partition bytes on rank {w.rank}")
    if not tr or any(t[2] != "device" for t in tr):
        out.append(f"memcheck transports {tr}")
    from dryad_amd.io.providers import provider_for
    provider_for("hbm://sweep_memcheck").delete("hbm://sweep_memcheck")
    return out


if __name__ == "__main__":
    main()
    # tear the process group down before the interpreter exits: gloo's threads torn down during
    # finalisation abort the process now and then ("terminate called without an active exception")
    from dryad_amd.parallel.comm import shutdown
    shutdown()

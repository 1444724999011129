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
        "terasort_where_take": (lambda c, W: c.FromStore(ts % W).Where(lambda r: r[0] < 16).Select(lambda r: r[0:4]),
                                False),
        "hash_partition": (lambda c, W: c.FromEnumerable(DATA).HashPartition(lambda x: x % 37, 4), False),
    }


def run(q, c, W):
    r = q(c, W)
    return r if isinstance(r, list) else list(r)


def main():
    w = init_world(device="cuda")
    W = w.size
    g = D.DryadLinqContext(platform="gpu")
    g.PartitionCount = W
    loc = D.DryadLinqContext(1)
    loc.LocalDebug = True
    bad = []
    for name, (q, ordered) in queries().items():
        got = run(q, g, W)
        if w.rank == 0:
            exp = run(q, loc, W)
            norm = (lambda x: [bytes(v) if isinstance(v, (bytes, bytearray, memoryview)) else v for v in x])
            a, b = norm(got), norm(exp)
            ok = a == b if ordered else sorted(a, key=repr) == sorted(b, key=repr)
            if not ok:
                bad.append(name)
            print(f"[sweep] {name}: {'ok' if ok else 'MISMATCH'} ({len(a)} rows)", flush=True)
    w.barrier()
    if w.rank == 0:
        assert not bad, bad
        print("SWEEP_OK", W, flush=True)


if __name__ == "__main__":
    main()

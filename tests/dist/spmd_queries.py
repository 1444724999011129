"""SPMD job run by every rank (launched by torch.distributed.run in tests/test_spmd.py).

Exercises the GPU executor's transport on CPU/gloo (or GPU/RCCL): cross shuffles (HashPartition,
GroupBy, Join, OrderBy range partitioning), merges (aggregates, Take), broadcasts (separators,
offsets) and host-store commits, each compared with the LocalDebug oracle on every rank."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import dryad_amd as D  # noqa: E402
from dryad_amd.parallel.comm import init_world, shutdown  # noqa: E402


def canon(xs):
    return sorted(xs, key=repr)


def main():
    dev = os.environ.get("SPMD_DEVICE", "cpu")
    w = init_world(device=dev)
    g = D.DryadLinqContext(platform="gpu")
    g._props["Device"] = dev
    g.PartitionCount = int(os.environ.get("SPMD_PARTS", str(w.size)))
    l = D.DryadLinqContext(1)
    l.LocalDebug = True
    data = [(i * 7919) % 1013 for i in range(3000)]
    pairs = [(i % 37, float(i)) for i in range(2000)]
    cases = [
        ("where_select", lambda c: c.FromEnumerable(data).Where(lambda x: x % 3 == 0).Select(lambda x: x + 1), False),
        ("groupby_decomp", lambda c: c.FromEnumerable(pairs).GroupBy(
            lambda t: t[0], lambda k, gr: (k, gr.Count(), gr.Sum(lambda t: t[1]), gr.Max(lambda t: t[1]))), False),
        ("groupby_groups", lambda c: c.FromEnumerable(data[:300]).GroupBy(lambda x: x % 5, lambda k, gr: (k, len(gr))), False),
        ("orderby", lambda c: c.FromEnumerable(data).OrderBy(lambda x: x), True),
        ("orderby_desc", lambda c: c.FromEnumerable(data).OrderByDescending(lambda x: x), True),
        ("hashpartition", lambda c: c.FromEnumerable(data).HashPartition(lambda x: x % 17), False),
        ("join", lambda c: c.FromEnumerable(pairs).Join(c.FromEnumerable(list(range(40))), lambda t: t[0],
                                                        lambda k: k, lambda t, k: (k, t[1])), False),
        ("distinct", lambda c: c.FromEnumerable(data).Select(lambda x: x % 100).Distinct(), False),
        ("take", lambda c: c.FromEnumerable(data).Take(10), True),
        ("indexed", lambda c: c.FromEnumerable(data[:100]).Select(lambda x, i: x * 0 + i), True),
        ("concat", lambda c: c.FromEnumerable([1, 2, 3]).Concat(c.FromEnumerable([4, 5])), True),
    ]
    for name, build, ordered in cases:
        a = list(build(l))
        b = list(build(g))
        ok = (a == b) if ordered else (canon(a) == canon(b))
        assert ok, f"rank {w.rank} {name}: {a[:8]} != {b[:8]}"
    # one k-means iteration: device_function Apply with a broadcast centroid table + merge Apply
    from dryad_amd.models.kmeans import step_query, POINT_T
    from dryad_amd.models.kmeans_cpu import gen_points
    cents = [tuple(r) for r in gen_points(0, 4, 5, 9).tolist()]
    km = lambda c: step_query(c.FromStore("gen://points?count=3000&partitions=%d&blobs=5&seed=9" % g.PartitionCount),  # noqa: E731
                              c.FromEnumerable(cents, dtype=POINT_T))
    a, b = list(km(l)), list(km(g))
    assert len(a) == len(b) == 4 and max(abs(x - y) for ra, rb in zip(a, b) for x, y in zip(ra, rb)) < 1e-5, \
        f"rank {w.rank} kmeans"
    for name, f in [("count", lambda c: c.FromEnumerable(data).Count()),
                    ("sum", lambda c: c.FromEnumerable(data).Sum()),
                    ("max", lambda c: c.FromEnumerable(data).Max())]:
        assert f(l) == f(g), f"rank {w.rank} {name}"
    w.barrier()
    if w.rank == 0:
        print("SPMD_OK", w.size, flush=True)
    shutdown()


if __name__ == "__main__":
    main()

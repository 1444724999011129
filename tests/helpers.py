"""Test helpers: the reference's oracle pattern (DryadLinqTests/*: every query runs on the cluster
and in LocalDebug and the results are compared, ApplyAndForkTests.cs:159-205; Validate.Check sorts
both sides, Utils.cs:305-374)."""
import os
import tempfile

import dryad_amd as D

_CTX = {}
# "cpu": the process executor (vertex hosts); "gpu": the SPMD GPU executor, n partitions on this
# process's GPU (tests/test_gpu_oracle_suites.py reruns the oracle suites that way)
MODE = "cpu"


def cluster_ctx(n=3, pool="thread"):
    key = (MODE, n, pool)
    c = _CTX.get(key)
    if c is None:
        if MODE == "gpu":
            c = D.DryadLinqContext(platform="gpu")
            c.PartitionCount = n
        else:
            c = D.DryadLinqContext(n)
            c._props["PoolKind"] = pool
            c._props["OutlierThresholdSeconds"] = None
        _CTX[key] = c
    return c


def local_ctx():
    c = D.DryadLinqContext(1)
    c.LocalDebug = True
    return c


def _norm(x):
    if isinstance(x, D.Grouping):
        return ("G", _norm(x.Key), tuple(_norm(e) for e in x))
    if isinstance(x, list):
        return tuple(_norm(e) for e in x)
    if isinstance(x, tuple):
        return tuple(_norm(e) for e in x)
    if isinstance(x, float):
        return round(x, 9)
    return x


def canon(seq, ordered=False):
    vals = [_norm(x) for x in seq]
    return vals if ordered else sorted(vals, key=repr)


def both(build, n=3, ordered=False, pool="thread"):
    """build(ctx) -> Query or scalar; asserts cluster == LocalDebug and returns the result."""
    a = build(local_ctx())
    b = build(cluster_ctx(n, pool))
    if hasattr(a, "node"):
        a, b = list(a), list(b)
        assert canon(a, ordered) == canon(b, ordered), f"\nLocalDebug: {canon(a, ordered)[:20]}\ncluster:    {canon(b, ordered)[:20]}"
        return b
    assert _norm(a) == _norm(b), f"LocalDebug {a!r} != cluster {b!r}"
    return b


def tmpdir():
    return tempfile.mkdtemp(prefix="dryad-test-")

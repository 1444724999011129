"""Partition-property bookkeeping of the planner (DataSetInfo.cs:91-799 analogue) and the
partitioner hash shared by host and device vertices."""
import struct

import dryad_amd as D
from dryad_amd.compiler.planner import compile_queries
from dryad_amd.runtime.vertex_ops import hash_port, stable_hash


def _ctx(parts=4):
    c = D.DryadLinqContext(2)
    c.PartitionCount = parts
    return c


def _range_ops(plan):
    return [op for s in plan.stages for op in s.ops if op.get("op") == "range_partition"]


def test_orderby_alone_may_split_ties():
    c = _ctx()
    q = c.FromEnumerable(list(range(100))).OrderBy(lambda x: x % 7)
    ops = _range_ops(compile_queries(c, [q]))
    assert ops and not any(op.get("keep_ties") for op in ops)


def test_orderby_then_groupby_same_key_keeps_ties():
    """GroupBy elides its shuffle after OrderBy on the same key, so the range partition must keep
    equal keys on one partition (the fused GPU OrderBy would otherwise split skewed runs)."""
    c = _ctx()
    key = lambda x: x % 7  # noqa: E731
    q = c.FromEnumerable(list(range(100))).OrderBy(key).GroupBy(key, lambda k, g: (k, g.Count()))
    plan = compile_queries(c, [q])
    ops = _range_ops(plan)
    assert ops and all(op.get("keep_ties") for op in ops)
    assert not any(op.get("op") == "hash_partition" for s in plan.stages for op in s.ops)


def test_orderby_then_groupby_other_key_reshuffles():
    c = _ctx()
    q = c.FromEnumerable(list(range(100))).OrderBy(lambda x: x % 7).GroupBy(lambda x: x % 5, lambda k, g: (k, g.Count()))
    plan = compile_queries(c, [q])
    assert not any(op.get("keep_ties") for op in _range_ops(plan))
    assert any(op.get("op") == "hash_partition" for s in plan.stages for op in s.ops)


def test_orderby_groupby_duplicates_match_oracle():
    data = [(i * 37) % 11 for i in range(5000)]
    key = lambda x: x  # noqa: E731
    c = _ctx(3)
    got = sorted(c.FromEnumerable(data).OrderBy(key).GroupBy(key, lambda k, g: (k, g.Count())))
    loc = D.DryadLinqContext(1)
    loc.LocalDebug = True
    exp = sorted(loc.FromEnumerable(data).OrderBy(key).GroupBy(key, lambda k, g: (k, g.Count())))
    assert got == exp


def test_stable_hash_canonical_values():
    # the device partitioner (csrc/kernels/stablehash.hip) mirrors these definitions
    assert stable_hash(3) == stable_hash(3.0)
    assert stable_hash(-0.0) == stable_hash(0.0) == stable_hash(0)
    nan_a = struct.unpack("<d", struct.pack("<Q", 0x7FF8000000000001))[0]
    assert stable_hash(float("nan")) == stable_hash(nan_a)
    assert stable_hash(float("inf")) != stable_hash(float("-inf"))
    assert stable_hash(True) == 1 and stable_hash(False) == 0
    assert 0 <= hash_port((1, "a", b"xy", 2.5), 1000) < 1000

"""Which stage pairs the GPU executor runs as a streamed shuffle (runtime/stream_shuffle.find):
a decomposable GroupBy / Distinct over a cross edge (partial side -> final side) and a repartition
written to a store (HashPartition -> record-wise -> ToStore); not a pair whose final side does
more than record-wise work before its output, nor a source with inputs.  CPU-only: plan shapes."""
import pytest

import dryad_amd as D
from dryad_amd.compiler.planner import compile_queries
from dryad_amd.runtime import stream_shuffle as SSH

SRC = "gen://records64?count=100000&partitions=4&keys=5000&seed=1"


@pytest.fixture
def ctx():
    c = D.DryadLinqContext(platform="gpu")
    c.PartitionCount = 4
    return c


def _find(ctx, q):
    plan = compile_queries(ctx, [q])
    return plan, SSH.find(plan)


def test_groupby_pair(ctx, tmp_path):
    q = ctx.FromStore(SRC).Where(lambda r: r[1] > 3).GroupBy(lambda r: r[0], lambda k, g: (k, g.Count()))
    plan, found = _find(ctx, q.ToStore(f"partfile://{tmp_path}/g"))
    assert len(found) == 1
    d = next(iter(found.values()))
    assert d.get("mode") is None and [o["op"] for o in plan.stages[d["a"]].ops][-1] == "hash_partition"


def test_distinct_pair(ctx, tmp_path):
    q = ctx.FromStore(SRC).Select(lambda r: r[0] % 97).Distinct()
    _, found = _find(ctx, q.ToStore(f"partfile://{tmp_path}/d"))
    assert len(found) == 1


def test_repartition_to_store(ctx, tmp_path):
    q = ctx.FromStore(SRC).Where(lambda r: r[2] % 3 != 0).HashPartition(lambda r: r[0], 4).Select(
        lambda r: (r[0], r[1] + 1))
    plan, found = _find(ctx, q.ToStore(f"partfile://{tmp_path}/r"))
    assert len(found) == 1
    d = next(iter(found.values()))
    assert d["mode"] == "repartition"
    assert [o["op"] for o in plan.stages[d["b"]].ops] == ["select", "output"]


def test_repartition_followed_by_an_aggregate_is_not_streamed(ctx, tmp_path):
    q = ctx.FromStore(SRC).HashPartition(lambda r: r[0], 4).OrderBy(lambda r: r[1])
    _, found = _find(ctx, q.ToStore(f"partfile://{tmp_path}/o"))
    assert not any(d.get("mode") == "repartition" for d in found.values())

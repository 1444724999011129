"""Which stages the GPU executor streams chunk by chunk (runtime/streaming.streamable): read ->
record-wise operators -> partfile write, over sources it can cut into chunks; anything with an
aggregate, an index overload, an HBM output or a non-chunkable source keeps whole partitions.
CPU-only: the decision needs no device."""
from types import SimpleNamespace

import pytest

import dryad_amd as D
from dryad_amd.compiler.planner import compile_queries
from dryad_amd.runtime import streaming as ST


def _runner(ctx):
    return SimpleNamespace(gpu_ok=True, ctx=ctx, skipped=set(), gang_stages=set())


def _stages(ctx, q):
    return compile_queries(ctx, [q]).stages


@pytest.fixture
def ctx():
    c = D.DryadLinqContext(platform="gpu")
    c.PartitionCount = 2
    c.StreamStages = True
    c.StreamChunkBytes = 1 << 16
    return c


def test_record_wise_to_partfile_streams(ctx, tmp_path):
    src = ctx.FromStore("gen://range?count=300000&partitions=2")
    q = src.Where(lambda x: x % 3 != 0).Select(lambda x: x * 2).ToStore(f"partfile://{tmp_path}/o")
    st = _stages(ctx, q)
    assert len(st) == 1
    plan = ST.streamable(_runner(ctx), st[0])
    assert plan is not None and plan["kind"] == "range" and plan["chunk"] == 1 << 16


def test_gen_rows_to_partfile_streams(ctx, tmp_path):
    q = ctx.FromStore("gen://terasort?records=1000&partitions=1&seed=1").ToStore(f"partfile://{tmp_path}/t")
    assert ST.streamable(_runner(ctx), _stages(ctx, q)[0])["kind"] == "terasort"


@pytest.mark.parametrize("case", ["groupby", "select_idx", "hbm_out", "points"])
def test_not_streamed(ctx, tmp_path, case):
    src = ctx.FromStore("gen://range?count=300000&partitions=2")
    if case == "groupby":
        q = src.GroupBy(lambda x: x % 7, lambda k, g: (k, g.Count())).ToStore(f"partfile://{tmp_path}/g")
    elif case == "select_idx":
        q = src.Select(lambda x, i: x + i).ToStore(f"partfile://{tmp_path}/i")
    elif case == "hbm_out":
        q = src.Select(lambda x: x + 1).ToStore("hbm://streaming_plan_test")
    else:
        q = ctx.FromStore("gen://points?count=1000&partitions=1&blobs=4&seed=1").ToStore(f"partfile://{tmp_path}/p")
    assert all(ST.streamable(_runner(ctx), s) is None for s in _stages(ctx, q))


def test_threshold_without_force(tmp_path):
    c = D.DryadLinqContext(platform="gpu")
    c.StreamChunkBytes = 1 << 20
    small = c.FromStore("gen://range?count=1000&partitions=1").Select(lambda x: x).ToStore(f"partfile://{tmp_path}/s")
    assert ST.streamable(_runner(c), _stages(c, small)[0]) is None            # 8 KB partition: whole
    big = c.FromStore("gen://range?count=1000000&partitions=1").Select(lambda x: x).ToStore(f"partfile://{tmp_path}/b")
    assert ST.streamable(_runner(c), _stages(c, big)[0]) is not None          # 8 MB > 1 MB chunks

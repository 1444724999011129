"""Bounded, chunk-streamed stages (runtime/streaming.py): read -> record-wise operators -> partfile
write, chunk by chunk, for every chunkable source (stored raw rows, stored fixed-width binary
records, gen://terasort, gen://records64, gen://range); the written tables must equal the
LocalDebug oracle, and the executor must report the chunks it streamed."""
import pytest

import dryad_amd as D

pytestmark = pytest.mark.gpu


def _ctx(chunk=1 << 20):
    c = D.DryadLinqContext(platform="gpu")
    c.StreamStages = True
    c.StreamChunkBytes = chunk
    return c


def _streamed(c):
    return c._get_executor().last_result.get("streamed") or {}


def test_gen_range_select_where_streams(tmp_path):
    c = _ctx(1 << 16)
    c.PartitionCount = 2
    out = f"partfile://{tmp_path}/r"
    c.FromStore("gen://range?count=300000&partitions=2").Where(lambda x: x % 3 != 0) \
        .Select(lambda x: x * 2 + 1).ToStore(out, delete_if_exists=True).SubmitAndWait()
    st = _streamed(c)
    assert st and all(v["chunks"] > 1 for v in st.values()), st
    got = sorted(D.DryadLinqContext(1).FromStore(out))
    assert got == sorted(x * 2 + 1 for x in range(300000) if x % 3 != 0)


def test_records64_projection_streams(tmp_path):
    c = _ctx(1 << 20)
    out = f"partfile://{tmp_path}/p"
    src = "gen://records64?count=200000&partitions=1&keys=1000&seed=9"
    c.FromStore(src).Where(lambda r: r[0] < 500).Select(lambda r: (r[0], r[1] + r[2])) \
        .ToStore(out, delete_if_exists=True).SubmitAndWait()
    assert _streamed(c)
    loc = D.DryadLinqContext(1)
    loc.LocalDebug = True
    exp = sorted(loc.FromStore(src).Where(lambda r: r[0] < 500).Select(lambda r: (r[0], r[1] + r[2])))
    assert sorted(D.DryadLinqContext(1).FromStore(out)) == exp


def test_stored_rows_roundtrip_streams(tmp_path):
    c = _ctx(8 << 20)
    a, b = f"partfile://{tmp_path}/a", f"partfile://{tmp_path}/b"
    c.FromStore("gen://terasort?records=400000&partitions=1&seed=3").ToStore(a, delete_if_exists=True).SubmitAndWait()
    assert _streamed(c)
    c2 = _ctx(8 << 20)
    c2.FromStore(a).Where(lambda r: r[0] < 128).ToStore(b, delete_if_exists=True).SubmitAndWait()
    st = _streamed(c2)
    assert st and list(st.values())[0]["chunks"] > 1
    loc = D.DryadLinqContext(1)
    loc.LocalDebug = True
    exp = [r for r in loc.FromStore("gen://terasort?records=400000&partitions=1&seed=3") if r[0] < 128]
    got = list(D.DryadLinqContext(1).FromStore(b))
    assert sorted(map(bytes, got)) == sorted(map(bytes, exp))

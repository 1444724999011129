"""Column bounds travel with a stored table: the GPU executor's partfile writer records each
integer column's [min, max] in the schema sidecar and a device read registers them, so a GroupBy
over the stored table packs by value width without a min / max pass."""
import json

import pytest
import torch

import dryad_amd as D

pytestmark = pytest.mark.gpu


def test_partfile_schema_keeps_column_bounds(tmp_path):
    from dryad_amd.gpu import stats as GST
    from dryad_amd.runtime.jobmanager import schema_path
    uri = "partfile://" + str(tmp_path / "r64.pt")
    g = D.DryadLinqContext(platform="gpu")
    g.PartitionCount = 2
    src = "gen://records64?count=200000&partitions=2&keys=5000&seed=3&cols=4"
    g.FromStore(src).Select(lambda r: (r[0], r[1] - 7, r[2])).ToStore(uri, delete_if_exists=True).SubmitAndWait()
    res0 = g._get_executor().last_result
    assert res0["fallbacks"] == [], res0["fallbacks"]
    sch = json.load(open(schema_path(str(tmp_path / "r64.pt"))))
    b = sch.get("bounds")
    assert b is not None and len(b) == 3, sch
    loc = D.DryadLinqContext(1)
    loc.LocalDebug = True
    rows = list(loc.FromStore(src).Select(lambda r: (r[0], r[1] - 7, r[2])))
    exp = [[min(x[j] for x in rows), max(x[j] for x in rows)] for j in range(3)]
    # bounds, not extremes: a column the generator declared keeps its declared range, a computed
    # one is measured exactly
    got_b = [b[f"Item{j + 1}"] for j in range(3)]
    assert all(lo <= e[0] and e[1] <= hi for (lo, hi), e in zip(got_b, exp)), (b, exp)
    assert got_b[1] == exp[1], (b, exp)
    # a device read of a part registers them on its columns
    from types import SimpleNamespace
    from dryad_amd.gpu.ops import OPS
    v = SimpleNamespace(partition=0, device=torch.device("cuda"), runner=None, stage=None)
    t = OPS["read"](dict(op="read", uri=uri), [], v)
    assert t.n > 0 and [GST.known(t.cols[f]) for f in sorted(b)] == [tuple(b[f]) for f in sorted(b)]
    got = sorted(g.FromStore(uri).GroupBy(lambda r: r[0], lambda k, grp: (k, grp.Count())))
    assert len(got) == len({x[0] for x in rows}) and sum(c for _, c in got) == len(rows)
    res = g._get_executor().last_result
    assert res["fallbacks"] == [], res["fallbacks"]


def test_columnar_result_to_host_table_stays_columnar():
    """A columnar device result written to host:// is DMA'd into pinned host columns (not turned
    into Python records) and read back to the device with its bounds."""
    from dryad_amd.gpu import stats as GST
    from dryad_amd.io.hosttable import HostColumns
    from dryad_amd.io.providers import provider_for
    g = D.DryadLinqContext(platform="gpu")
    src = "gen://records64?count=300000&partitions=1&keys=7000&seed=9&cols=3"
    g.FromStore(src).ToStore("host://cols_src", delete_if_exists=True).SubmitAndWait()
    h = provider_for("host://cols_src").get("host://cols_src")["local"][0]
    assert isinstance(h, HostColumns) and h.n == 300000
    t = h.to_device(torch.device("cuda"))
    assert GST.known(t.cols[list(t.cols)[0]]) == (0, 6999)
    got = sorted(g.FromStore("host://cols_src").GroupBy(lambda r: r[0], lambda k, grp: (k, grp.Count())))
    loc = D.DryadLinqContext(1)
    loc.LocalDebug = True
    assert got == sorted(loc.FromStore(src).GroupBy(lambda r: r[0], lambda k, grp: (k, grp.Count())))

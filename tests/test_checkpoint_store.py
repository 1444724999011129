"""runtime/checkpoint.StageCheckpoint: vertex outputs persisted raw through the native part writer
(pieces round-robin over several data files) and loaded back piece by piece; every output kind."""
import os

import torch

from dryad_amd.gpu.table import DeviceTable, Ported, PortTables, Shape
from dryad_amd.runtime import checkpoint as CK


def _same(a, b):
    if isinstance(a, DeviceTable):
        assert isinstance(b, DeviceTable) and a.n == b.n and a.shape == b.shape
        assert a.to_objects() == b.to_objects()
        return
    assert a == b


def _strings_table(n):
    words = [("w%d" % i) * (i % 5) for i in range(n)]
    enc = [w.encode() for w in words]
    ln = torch.tensor([len(e) for e in enc], dtype=torch.int64)
    off = torch.cumsum(ln, 0) - ln
    heap = torch.frombuffer(bytearray(b"".join(enc)), dtype=torch.uint8).clone()
    return DeviceTable(n, Shape("tuple", ["Item1", "Item2"]),
                       {"Item1": torch.arange(n, dtype=torch.int64), "Item2": off, "Item2#len": ln},
                       strs={"Item2": heap})


def test_round_trip_of_every_output_kind(tmp_path, monkeypatch):
    monkeypatch.setattr(CK, "PIECE", 4096)            # many pieces over several data files
    ck = CK.StageCheckpoint(str(tmp_path), "job0001-x")
    cols = DeviceTable.from_columns({"a": torch.arange(5000, dtype=torch.int64) * 7,
                                     "b": torch.rand(5000, dtype=torch.float32)}, Shape("tuple", ["a", "b"]))
    rows = DeviceTable.from_rows(torch.randint(0, 255, (3000, 24), dtype=torch.uint8), 0, 10)
    strs = _strings_table(2000)
    ported = Ported(cols, [0, 1000, 5000], None)
    ports = PortTables([strs, [("x", 1), ("y", 2)], None])
    values = [cols, rows, strs, ported, ports, None, [(1, "a"), (2, "b")], cols.slice(0, 0)]
    for p, v in enumerate(values):
        assert ck.save(3, p, v) > 0
        assert ck.has(3, p)
    files = os.listdir(os.path.join(ck.dir, "s3"))
    assert any(f.startswith("p0.d7") for f in files), files       # 80 KB in 4 KB pieces: 8 data files
    for p, v in enumerate(values):
        got = ck.load(3, p, "cpu")
        if isinstance(v, Ported):
            assert got.offsets == v.offsets and got.order == v.order
            _same(v.table, got.table)
        elif isinstance(v, PortTables):
            _same(v.tables[0], got.tables[0])
            assert got.tables[1] == v.tables[1] and got.tables[2] is None
        else:
            _same(v, got)
    ck.drop(3, 0)
    assert not ck.has(3, 0) and not [f for f in os.listdir(os.path.join(ck.dir, "s3")) if f.startswith("p0.")]


def test_nbytes_and_budget(tmp_path):
    ck = CK.StageCheckpoint(str(tmp_path), "job0002-y", budget=1000)
    t = DeviceTable.from_columns({"a": torch.arange(100, dtype=torch.int64)}, Shape("scalar", ["a"]))
    assert CK.StageCheckpoint.nbytes(t) == 800 and ck.budget == 1000
    ck.save(0, 0, t)
    assert ck.used == 800


def _job(tmp_path, budget):
    import dryad_amd as D
    g = D.DryadLinqContext(platform="gpu")
    g._props["Device"] = "cpu"
    g.PartitionCount = 2
    g.PersistStageOutputs = str(tmp_path / "ck")
    if budget is not None:
        g.CheckpointBudgetBytes = budget
    q = g.FromEnumerable([(i % 13, i) for i in range(2000)]).GroupBy(
        lambda t: t[0], lambda k, grp: (k, grp.Count(), grp.Sum(lambda t: t[1])))
    got = sorted(q)
    return g, got


def test_executor_persists_per_stage_and_skips_past_the_budget(tmp_path):
    g, got = _job(tmp_path, None)
    assert got == sorted((k, sum(1 for i in range(2000) if i % 13 == k), sum(i for i in range(2000) if i % 13 == k))
                         for k in range(13))
    res = g._get_executor().last_result
    per = res["persist"]
    assert per and all("ms" in v and v["bytes"] > 0 for v in per.values()), per
    evs = [e.get("ev") for e in res["events"]]
    assert "stage_persisted" in evs, evs
    g2, got2 = _job(tmp_path, 1)
    assert got2 == got
    res2 = g2._get_executor().last_result
    assert res2["persist"] and all(v.get("skipped") == "budget" for v in res2["persist"].values()), res2["persist"]
    assert "persist_skipped" in [e.get("ev") for e in res2["events"]]
